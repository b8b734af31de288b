"""GPU parity of the horizontal co-occurrence counts: the level-2 pair gram counted from the
transaction CSR — row by row in LDS (csrc/kernels/pairrows.hip, the default) and by scattered
atomics (csrc/kernels/cooc.hip, test hook pair_rows=0) — checked against a numpy one-hot Gram
(float64 BLAS, exact) and against the bitmap bit-GEMM of the same shard; and the miner with the
level-2 method forced each way producing the same trie (content digest)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _onehot(ptr, items, n_tx, n_items):
    X = np.zeros((n_tx, n_items), dtype=np.float64)
    rows = np.repeat(np.arange(n_tx), np.diff(ptr))
    X[rows, items] = 1.0
    return X


def _miner(gpu_mod, ptr, items, n_items):
    import torch
    g = gpu_mod.GpuMiner(0, 1 << 28, torch.cuda.current_stream().cuda_stream or 0)
    g.load_csr(ptr, items, n_items)
    return g


@pytest.fixture(params=["rows", "atomic"])
def method(request, monkeypatch):
    monkeypatch.setenv("KMLS_TEST_HOOKS", "pair_rows=1" if request.param == "rows" else "pair_rows=0")
    return request.param


@pytest.mark.parametrize("shape,ms,n_tx,ld_pad", [("tiny", 0.02, None, 0), ("ds2", 0.05, 1500, 3),
                                                  ("ds_dense", 0.05, None, 0),
                                                  ("ds2_weak", 0.01, 4000, 1)])
def test_cooc_vs_numpy(gpu_mod, method, shape, ms, n_tx, ld_pad):
    import torch
    from kubernetes_machine_learning_server_amd.data.synthetic import generate
    tx = generate(shape, seed=7, n_tx=n_tx)
    g = _miner(gpu_mod, tx.tx_ptr, tx.items, tx.n_items)
    counts = np.bincount(tx.items, minlength=tx.n_items).astype(np.uint32)
    F = g.select(counts, tx.n_tx, ms)
    ids = np.asarray(g.frequent()[0])
    st = g.cooc_stats()
    X = _onehot(tx.tx_ptr, tx.items, tx.n_tx, tx.n_items)[:, ids]
    k = X.sum(1).astype(np.int64)
    assert st["pairs"] == int((k * (k - 1) // 2).sum()) and st["max_k"] == int(k.max())
    ld = F + ld_pad
    gram = torch.full((F, ld), 7, dtype=torch.int32, device="cuda")  # stale: the call zeroes it
    torch.cuda.synchronize()
    assert g.pair_counts_csr(gram.data_ptr(), ld)
    g.synchronize()
    got = np.triu(gram.cpu().numpy()[:, :F].astype(np.int64), 1)
    ref = np.triu(np.rint(X.T @ X).astype(np.int64), 1)
    np.testing.assert_array_equal(got, ref)


def test_cooc_large_vocab_matches_bit_gemm(gpu_mod, method):
    """1M-item vocabulary (the frequent bit-mask filter) and > 2^16 transactions: equal to the
    popcount bit-GEMM over the shard's bitmaps."""
    import torch
    T, I = 300_000, 1_000_000
    ptr, items = gpu_mod.synth_transactions(T, I, 30.0, 2000, 0.85, 0.85, 5)
    g = _miner(gpu_mod, ptr, items, I)
    counts = np.bincount(items, minlength=I).astype(np.uint32)
    F = g.select(counts, T, 5e-4)
    assert F > 64  # the LDS head table and the global atomics both used
    Wp = g.words_local()
    bm = torch.zeros((F, Wp), dtype=torch.int64, device="cuda")
    ref = torch.zeros((F, F), dtype=torch.int32, device="cuda")
    got = torch.zeros((F, F), dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    g.encode_bitmaps(bm.data_ptr(), Wp, 0)
    g.pair_counts(bm.data_ptr(), Wp, ref.data_ptr(), False)
    assert g.pair_counts_csr(got.data_ptr(), F)
    g.synchronize()
    iu = np.triu_indices(F, 1)
    r, o = ref.cpu().numpy()[iu], got.cpu().numpy()[iu]
    assert r.sum() > 0
    np.testing.assert_array_equal(o, r)


def test_cooc_declines_long_transactions(gpu_mod, method):
    """A transaction with more frequent items than the LDS entry buffer: the atomic count
    declines (gram untouched); the row count takes it (its row is sorted in place)."""
    import torch
    n_items = 2100
    rows = [np.arange(n_items, dtype=np.int32)] + [np.array([1, 2, 3], np.int32)] * 50
    ptr = np.concatenate([[0], np.cumsum([len(r) for r in rows])]).astype(np.int64)
    items = np.concatenate(rows).astype(np.int32)
    g = _miner(gpu_mod, ptr, items, n_items)
    counts = np.bincount(items, minlength=n_items).astype(np.uint32)
    F = g.select(counts, len(rows), 0.0)
    assert F == n_items and g.cooc_stats()["max_k"] == n_items
    gram = torch.full((F, F), 5, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    if method == "atomic":
        assert not g.pair_counts_csr(gram.data_ptr(), F)
        g.synchronize()
        assert int(gram[0, 1].item()) == 5
        return
    assert g.pair_counts_csr(gram.data_ptr(), F)
    g.synchronize()
    ids = np.asarray(g.frequent()[0])
    X = _onehot(ptr, items, len(rows), n_items)[:, ids]
    got = np.triu(gram.cpu().numpy().astype(np.int64), 1)
    np.testing.assert_array_equal(got, np.triu(np.rint(X.T @ X).astype(np.int64), 1))


def test_txdp_level2_method_same_trie(gpu_mod, monkeypatch):
    """mine_txdp (world 1) with level 2 forced through the horizontal count and through the
    bit-GEMM: the same itemsets and supports (content digest)."""
    T, I = 200_000, 50_000
    ptr, items = gpu_mod.synth_transactions(T, I, 25.0, 300, 0.9, 0.85, 9)
    out = {}
    for hook in ("cooc=2", "cooc=0"):
        monkeypatch.setenv("KMLS_TEST_HOOKS", hook)
        g = gpu_mod.GpuMiner(0, 1 << 30, 0)
        g.load_csr(ptr, items, I)
        r = g.mine_txdp(None, T, 1e-3)
        out[hook] = r
        assert r["stats"]["level2_method"] == ("cooc" if hook == "cooc=2" else "gram_popcount")
    a, b = out["cooc=2"], out["cooc=0"]
    assert a["stats"]["n_itemsets"] == b["stats"]["n_itemsets"] > 0
    da = gpu_mod.trie_digest(a["parent"], a["item"], a["count"], a["depth"])
    db = gpu_mod.trie_digest(b["parent"], b["item"], b["count"], b["depth"])
    assert da["digest"] == db["digest"] and da["per_depth"] == db["per_depth"]


def test_cooc_refuses_after_frequent_subset(gpu_mod):
    """use_frequent_subset leaves the rank tables on the full selection: the CSR-driven pair
    count and the rule map refuse (an F-row gram would be written past its end otherwise), the
    cost model declines, and a fresh select() restores them."""
    import torch
    from kubernetes_machine_learning_server_amd.data.synthetic import generate
    tx = generate("ds2", seed=7, n_tx=1500)
    g = _miner(gpu_mod, tx.tx_ptr, tx.items, tx.n_items)
    counts = np.bincount(tx.items, minlength=tx.n_items).astype(np.uint32)
    F = g.select(counts, tx.n_tx, 0.05)
    assert F > 4 and not g.subset_active()
    g.use_frequent_subset(np.arange(0, F, 2, dtype=np.int64))
    assert g.subset_active()
    gram = torch.zeros((F, F), dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    for call in (lambda: g.pair_counts_csr(gram.data_ptr(), F), lambda: g.cooc_stats(),
                 lambda: g.rule_map_from_gram(gram.data_ptr(), F, 1)):
        with pytest.raises(Exception, match="use_frequent_subset"):
            call()
    assert not g.cooc_preferred()
    assert g.select(counts, tx.n_tx, 0.05) == F and not g.subset_active()
    assert g.pair_counts_csr(gram.data_ptr(), F)
    g.cooc_check()


def test_cooc_flags_duplicate_rows(gpu_mod, method):
    """A row holding one frequent item twice breaks load_csr's precondition: the horizontal
    counts flag it (cooc_check / the row count raise) instead of silently double-counting."""
    import torch
    rows = [np.array([1, 2, 2, 3], np.int32)] + [np.array([1, 2, 3], np.int32)] * 20
    ptr = np.concatenate([[0], np.cumsum([len(r) for r in rows])]).astype(np.int64)
    items = np.concatenate(rows).astype(np.int32)
    g = _miner(gpu_mod, ptr, items, 8)
    counts = np.bincount(items, minlength=8).astype(np.uint32)
    F = g.select(counts, len(rows), 0.5)
    gram = torch.zeros((F, F), dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    if method == "rows":
        with pytest.raises(Exception, match="twice"):
            g.pair_counts_csr(gram.data_ptr(), F)
        return
    assert g.pair_counts_csr(gram.data_ptr(), F)
    with pytest.raises(Exception, match="duplicate"):
        g.cooc_check()


def test_pair_rows_long_rows_large_vocab(gpu_mod):
    """A >= 64k-item vocabulary (the LDS-mask filter) whose rows hold more frequent items than
    the 16-entry register sort (in-place path): the row count equals the numpy Gram."""
    import torch
    rng = np.random.default_rng(3)
    T, I, hot = 70_000, 100_000, 48
    rows = []
    for t in range(T):
        r = rng.choice(I - hot, 6, replace=False)
        if t % 20 == 0:
            r = np.concatenate([r, I - hot + rng.choice(hot, 24, replace=False)])
        rows.append(np.sort(r))
    ptr = np.zeros(T + 1, np.int64)
    ptr[1:] = np.cumsum([len(r) for r in rows])
    items = np.concatenate(rows).astype(np.int32)
    g = _miner(gpu_mod, ptr, items, I)
    counts = np.bincount(items, minlength=I).astype(np.uint32)
    F = g.select(counts, T, 500 / T)
    assert F >= hot
    gram = torch.zeros((F, F), dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    assert g.pair_counts_csr(gram.data_ptr(), F)
    g.synchronize()
    ids = np.asarray(g.frequent()[0])
    col = np.full(I, -1, np.int64)
    col[ids] = np.arange(F)
    X = np.zeros((T, F), dtype=np.float64)  # one-hot over the frequent items only
    rix = np.repeat(np.arange(T), np.diff(ptr))
    keep = col[items] >= 0
    X[rix[keep], col[items][keep]] = 1.0
    got = np.triu(gram.cpu().numpy().astype(np.int64), 1)
    np.testing.assert_array_equal(got, np.triu(np.rint(X.T @ X).astype(np.int64), 1))


def test_txdp_long_rows_take_the_mfma_gram(gpu_mod, monkeypatch):
    """Long bitmap rows (>= 4,096 words: 300k transactions) with level 2 on the bit-GEMM: the
    miner picks the masked-FP4 MFMA gram by itself (gram_mfma.hip, not forced by an option) and
    the trie equals the C++ miner's by content digest."""
    T, I = 300_000, 400
    ptr, items = gpu_mod.synth_transactions(T, I, 12.0, 20, 0.9, 0.85, 3)
    ms = 0.01
    monkeypatch.setenv("KMLS_TEST_HOOKS", "cooc=0")
    g = gpu_mod.GpuMiner(0, 1 << 30, 0)
    g.load_csr(ptr, items, I)
    r = g.mine_txdp(None, T, ms)
    assert r["stats"]["level2_method"] == "gram_mfma"
    d = gpu_mod.trie_digest(r["parent"], r["item"], r["count"], r["depth"])
    ref = gpu_mod.mine_cpu(ptr, items, I, ms, 0)
    want = gpu_mod.trie_digest(ref["parent"], ref["item"], ref["count"], ref["depth"])
    assert d["per_depth"][2] > 0 and d["digest"] == want["digest"]
