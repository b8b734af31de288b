"""GPU numerics/parity tests of the HIP kernels (run on a real MI355X via gpurun).

Every kernel is checked against an independent CPU reference of the same op: pair counts vs a
numpy one-hot Gram (fp64/int64), the full miner vs the C++ CPU miner (itself checked against
the mlxtend-faithful oracle in test_miner_cpu.py), the serve kernel vs the C++ matcher.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _trie_dict(r):
    par, it, cnt = r["parent"], r["item"], r["count"]
    memo = []
    out = {}
    for n in range(len(it)):
        s = (memo[par[n]] if par[n] >= 0 else frozenset()) | {int(it[n])}
        memo.append(s)
        out[s] = int(cnt[n])
    return out


def _digest(gpu_mod, r):
    return gpu_mod.trie_digest(r["parent"], r["item"], r["count"], r["depth"])


def assert_same_itemsets(gpu_mod, r, c):
    """Content equality of two tries: (itemset, support) multiset digest + per-size counts."""
    dr, dc = _digest(gpu_mod, r), _digest(gpu_mod, c)
    assert dr["per_depth"] == dc["per_depth"]
    assert dr["digest"] == dc["digest"]


def _onehot(tx):
    X = np.zeros((tx.n_tx, tx.n_items), dtype=np.int64)
    for t in range(tx.n_tx):
        X[t, tx.items[tx.tx_ptr[t]:tx.tx_ptr[t + 1]]] = 1
    return X


@pytest.mark.parametrize("use_mfma", [False, True])  # popcount bit-GEMM / masked-FP4 MFMA gram
@pytest.mark.parametrize("shape,ms,n_tx", [("tiny", 0.02, None), ("ds2_weak", 0.03, None),
                                             ("tiny", 0.01, 5000), ("ds2", 0.05, 777),
                                             ("ds2_weak", 0.03, 70000)])
def test_pair_gram_vs_numpy(gpu_mod, shape, ms, n_tx, use_mfma):
    import torch
    from kubernetes_machine_learning_server_amd.data.synthetic import generate
    tx = generate(shape, seed=11, n_tx=n_tx)
    # run the miner on torch's current stream so torch allocations/fills are ordered with it
    g = gpu_mod.GpuMiner(0, 1 << 28, torch.cuda.current_stream().cuda_stream or 0)
    g.load_csr(tx.tx_ptr, tx.items, tx.n_items)
    cnt = torch.zeros(tx.n_items, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    g.item_support(cnt.data_ptr())
    g.synchronize()
    host = cnt.cpu().numpy().view(np.uint32)
    X = _onehot(tx)
    np.testing.assert_array_equal(host, X.sum(0))
    F = g.select(host, tx.n_tx, ms)
    ids, counts, minsup = g.frequent()
    Wp = g.words_local()
    bm = torch.zeros((max(F, 1), Wp), dtype=torch.int64, device="cuda")
    gram = torch.zeros((F, F), dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()  # the fills ran on torch's stream
    g.encode_bitmaps(bm.data_ptr(), Wp, 0)
    g.pair_counts(bm.data_ptr(), Wp, gram.data_ptr(), use_mfma)
    g.synchronize()
    got = np.triu(gram.cpu().numpy().astype(np.int64), 1)
    Xf = X[:, ids]
    # float64 BLAS product: exact (counts < 2^53) and seconds instead of numpy's int64 loop
    ref = np.triu(np.rint(Xf.T.astype(np.float64) @ Xf.astype(np.float64)).astype(np.int64), 1)
    np.testing.assert_array_equal(got, ref)
    # bitmap rows popcount == supports
    pc = np.array([bin(int(w) & (2**64 - 1)).count("1") for w in bm.cpu().numpy().ravel()])
    np.testing.assert_array_equal(pc.reshape(max(F, 1), Wp).sum(1)[:F], counts)


def test_pair_gram_fp4_exact_past_2_24_transactions(gpu_mod):
    """FP4 operands accumulate in f32, exact only below 2^24 per block: with more transactions
    than that the split-K must keep every block's slice under it.  Checked against the popcount
    gram (integer arithmetic) on 17M transactions."""
    import torch
    T, I = (1 << 24) + 4099, 300
    ptr, items = gpu_mod.synth_transactions(T, I, 3.0, 4, 0.9, 0.85, 21)
    g = gpu_mod.GpuMiner(0, 1 << 30, torch.cuda.current_stream().cuda_stream or 0)
    g.load_csr(ptr, items, I)
    counts = np.bincount(items, minlength=I).astype(np.uint32)
    F = g.select(counts, T, 0.001)
    Wp = g.words_local()
    bm = torch.zeros((F, Wp), dtype=torch.int64, device="cuda")
    ref = torch.zeros((F, F), dtype=torch.int32, device="cuda")
    got = torch.zeros((F, F), dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    g.encode_bitmaps(bm.data_ptr(), Wp, 0)
    g.pair_counts(bm.data_ptr(), Wp, ref.data_ptr(), False)
    g.pair_counts(bm.data_ptr(), Wp, got.data_ptr(), True)
    g.synchronize()
    iu = np.triu_indices(F, 1)
    r, o = ref.cpu().numpy()[iu], got.cpu().numpy()[iu]
    assert r.max() > (1 << 24) // 64  # counts large enough that f32 rounding would show
    np.testing.assert_array_equal(o, r)


@pytest.mark.parametrize("fused", ["1", "0"])
@pytest.mark.parametrize("use_mfma", [False, True])
@pytest.mark.parametrize("shape,ms", [("tiny", 0.05), ("tiny", 0.02), ("ds2_weak", 0.05),
                                      ("ds2_weak", 0.03), ("ds2", 0.07), ("ds2", 0.05),
                                      ("ds_dense", 0.05)])
def test_gpu_miner_matches_cpu(gpu_mod, shape, ms, use_mfma, fused, monkeypatch):
    from kubernetes_machine_learning_server_amd.data.synthetic import generate
    monkeypatch.setenv("KMLS_TEST_HOOKS", f"fused_levels={fused}")
    tx = generate(shape, seed=5)
    g = gpu_mod.GpuMiner(0, 1 << 31, 0)
    g.load_csr(tx.tx_ptr, tx.items, tx.n_items)
    r = g.mine(ms, mfma=use_mfma)
    path = r["stats"]["levels_path"]
    assert path.startswith("fused") if fused == "1" else path == "chunked", r["stats"]
    c = gpu_mod.mine_cpu(tx.tx_ptr, tx.items, tx.n_items, ms)
    assert r["stats"]["n_itemsets"] == c["stats"]["n_itemsets"]
    assert r["stats"]["max_depth"] == c["stats"]["max_depth"]
    assert_same_itemsets(gpu_mod, r, c)
    if c["stats"]["n_itemsets"] < 300_000:
        assert _trie_dict(r) == _trie_dict(c)


def test_compact_download_widths(gpu_mod):
    """The resident path streams the trie to the host at the narrowest exact widths
    (kernels.hpp HostTrie); the first call (pinned arrays sized from a previous call) overflows
    them and falls back to the full-width copy — both must hold the same trie."""
    from kubernetes_machine_learning_server_amd.data.synthetic import generate
    tx = generate("ds2_weak", seed=4)
    g = gpu_mod.GpuMiner(0, 1 << 31, 0)
    g.load_csr(tx.tx_ptr, tx.items, tx.n_items)
    first = g.mine(0.03)
    second = g.mine(0.03)
    c = gpu_mod.mine_cpu(tx.tx_ptr, tx.items, tx.n_items, 0.03)
    assert second["stats"]["levels_path"] == "fused-resident"
    if first["stats"]["n_itemsets"] > (1 << 16):  # first call's host arrays were too small
        assert first["parent"].dtype == np.int64 and first["count"].dtype == np.uint32
    assert second["parent"].dtype == np.int32
    assert second["item"].dtype == np.uint16 and second["count"].dtype == np.uint16
    for r in (first, second):
        assert _trie_dict(r) == _trie_dict(c)
        np.testing.assert_array_equal(r["depth"], first["depth"])


def test_gpu_miner_max_len_and_pairs(gpu_mod):
    from kubernetes_machine_learning_server_amd.data.synthetic import generate
    tx = generate("ds2_weak", seed=2)
    g = gpu_mod.GpuMiner(0, 1 << 30, 0)
    g.load_csr(tx.tx_ptr, tx.items, tx.n_items)
    for ml in (1, 2, 3):
        r = g.mine(0.03, max_len=ml)
        c = gpu_mod.mine_cpu(tx.tx_ptr, tx.items, tx.n_items, 0.03, max_len=ml)
        assert _trie_dict(r) == _trie_dict(c)
    r = g.mine(0.03, pairs_only=True)
    assert int(r["depth"].max()) <= 2


def test_gpu_miner_chunked_levels(gpu_mod, monkeypatch):
    """Force many candidates per level (multi-chunk path) on a larger synthetic set."""
    from kubernetes_machine_learning_server_amd.data.synthetic import generate
    monkeypatch.setenv("KMLS_TEST_HOOKS", "fused_levels=0")
    tx = generate("ds_dense", seed=9)
    g = gpu_mod.GpuMiner(0, 8 << 30, 0)
    g.load_csr(tx.tx_ptr, tx.items, tx.n_items)
    r = g.mine(0.045)
    c = gpu_mod.mine_cpu(tx.tx_ptr, tx.items, tx.n_items, 0.045)
    assert r["stats"]["n_itemsets"] == c["stats"]["n_itemsets"]
    assert_same_itemsets(gpu_mod, r, c)


def test_fused_levels_repeat_and_small_arena(gpu_mod, monkeypatch):
    """Repeated calls (epoch-tagged look-back state, persistent output buffers, streamed
    download sized from the previous call) and the fallback when the arena is too small."""
    from kubernetes_machine_learning_server_amd.data.synthetic import generate
    tx = generate("ds_dense", seed=3)
    c = gpu_mod.mine_cpu(tx.tx_ptr, tx.items, tx.n_items, 0.05)
    g = gpu_mod.GpuMiner(0, 4 << 30, 0)
    g.load_csr(tx.tx_ptr, tx.items, tx.n_items)
    keep = []
    for i in range(4):
        r = g.mine(0.05)
        assert r["stats"]["levels_path"] == "fused-resident", r["stats"]
        assert r["stats"]["n_itemsets"] == c["stats"]["n_itemsets"]
        keep.append(r)  # results stay valid while later calls run (pinned buffers not reused)
    for r in keep:
        assert_same_itemsets(gpu_mod, r, c)
    monkeypatch.setenv("KMLS_TEST_HOOKS", "fused_bump_mb=64")  # device allocations overflow mid-way
    small = gpu_mod.GpuMiner(0, 2 << 30, 0)
    small.load_csr(tx.tx_ptr, tx.items, tx.n_items)
    r = small.mine(0.05)
    assert "fallback: device overflow code 1" in r["stats"]["levels_path"], r["stats"]
    assert r["stats"]["n_itemsets"] == c["stats"]["n_itemsets"]
    assert_same_itemsets(gpu_mod, r, c)


def test_gpu_serve_matches_cpu(gpu_mod):
    from kubernetes_machine_learning_server_amd.data.synthetic import generate
    from kubernetes_machine_learning_server_amd.serve.index import build_index_from_trie
    tx = generate("ds2_weak", seed=4)
    c = gpu_mod.mine_cpu(tx.tx_ptr, tx.items, tx.n_items, 0.03, pairs_only=True)
    idx = build_index_from_trie(c["parent"], c["item"], c["count"], c["depth"], tx.n_tx,
                                tx.n_items)
    host = idx.native()
    gidx = gpu_mod.GpuRuleIndex(0, host)
    rng = np.random.default_rng(0)
    B = 512
    lens = rng.integers(1, 8, size=B)
    lens[7], lens[8], lens[9] = 70, 130, 300  # multi-pass seed gather; > 256 seeds → host (-2)
    q_ptr = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    keys = np.nonzero(idx.is_key)[0]
    seeds = np.where(rng.random(q_ptr[-1]) < 0.8, rng.choice(keys, q_ptr[-1]),
                     rng.integers(0, tx.n_items, q_ptr[-1])).astype(np.int32)
    seeds[q_ptr[5]:q_ptr[6]] = -1  # a query with no known seed
    for k in (1, 10, 25):
        ids, n = gidx.query_batch(q_ptr, seeds, k)
        cids, cn = host.query_batch(q_ptr, seeds, k)
        ok = n != -2  # the host answers the overflow queries (MicroBatcher does this)
        assert (n[~ok] == -2).all() and ok.sum() >= B - 2
        assert n[9] == -2  # 300 seeds
        np.testing.assert_array_equal(n[ok], cn[ok])
        np.testing.assert_array_equal(ids[ok], cids[ok])
    for B in (1, 3, 5):  # partial last block (4 queries per block)
        ids, n = gidx.query_batch(q_ptr[:B + 1], seeds[:q_ptr[B]], 10)
        cids, cn = host.query_batch(q_ptr[:B + 1], seeds[:q_ptr[B]], 10)
        np.testing.assert_array_equal(n, cn)
        np.testing.assert_array_equal(ids, cids)


def _long_row_index(rng, n_items=3000, n_keys=150, max_row=2500, n_scores=40, sort_rows=True):
    """Rule index with rows of 100..max_row entries and few distinct scores (many ties, the
    same consequent at different scores in different rows)."""
    from kubernetes_machine_learning_server_amd.serve.index import RuleIndexData
    keys = rng.choice(n_items, n_keys, replace=False)
    row_ptr = np.zeros(n_items + 1, np.int64)
    rows = {}
    for kk in keys:
        n = int(rng.integers(100, max_row))
        cons = rng.choice(np.setdiff1d(np.arange(n_items), [kk]), n, replace=False)
        sc = rng.integers(1, n_scores + 1, n).astype(np.float64) / 1000.0
        if sort_rows:
            o = np.argsort(-sc, kind="stable")
            cons, sc = cons[o], sc[o]
        rows[int(kk)] = (cons.astype(np.int32), sc)
    for i in range(n_items):
        row_ptr[i + 1] = row_ptr[i] + (len(rows[i][0]) if i in rows else 0)
    cons = np.concatenate([rows[i][0] for i in sorted(rows)])
    score = np.concatenate([rows[i][1] for i in sorted(rows)])
    is_key = np.zeros(n_items, np.uint8)
    is_key[keys] = 1
    return RuleIndexData(n_items, row_ptr, cons, score, is_key, None), keys


@pytest.mark.parametrize("sort_rows", [True, False])
def test_gpu_serve_long_rows(gpu_mod, sort_rows):
    """Long-merge queries (rows of thousands of entries: the HBM-scale indexes) on the
    workgroup kernel: threshold-pruned merge + first positions completed from earlier rows'
    suffixes == the C++ matcher, ties included.  Unsorted rows (a reference-format pickle)
    must not use the pruning: those queries go to the host (-2)."""
    rng = np.random.default_rng(3)
    idx, keys = _long_row_index(rng, sort_rows=sort_rows)
    host = idx.native()
    gidx = gpu_mod.GpuRuleIndex(0, host)
    B = 300
    lens = rng.integers(1, 13, size=B)
    lens[0], lens[1] = 200, 256  # many long rows in one query
    q_ptr = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    seeds = np.where(rng.random(q_ptr[-1]) < 0.85, rng.choice(keys, q_ptr[-1]),
                     rng.integers(0, idx.n_items, q_ptr[-1])).astype(np.int32)
    seeds[q_ptr[2] + 1] = seeds[q_ptr[2]]  # a repeated seed
    for k in (1, 10, 40):
        ids, n = gidx.query_batch(q_ptr, seeds, k)
        cids, cn = host.query_batch(q_ptr, seeds, k)
        ok = n != -2
        if sort_rows:
            assert ok.sum() >= B - 2, (n == -2).sum()
        else:
            assert (~ok).sum() >= B // 2  # long merges without pruning: host path
        np.testing.assert_array_equal(n[ok], cn[ok])
        np.testing.assert_array_equal(ids[ok], cids[ok])


def test_dist_miner_world1(gpu_mod):
    from kubernetes_machine_learning_server_amd.data.synthetic import generate
    from kubernetes_machine_learning_server_amd.parallel.dist_miner import DistMiner
    tx = generate("ds2_weak", seed=1)
    dm = DistMiner(tx.tx_ptr, tx.items, tx.n_items, 0.03)
    st = dm.step()["stats"]
    c = gpu_mod.mine_cpu(tx.tx_ptr, tx.items, tx.n_items, 0.03)
    assert st["global_itemsets"] == c["stats"]["n_itemsets"]


def test_dist_protocol_path_on_gpu(gpu_mod):
    """The multi-GPU protocol code path (torch HBM buffers, gram-based partition, owned-mask
    DFS) at world size 1 on the real device."""
    from kubernetes_machine_learning_server_amd.data.synthetic import generate
    from kubernetes_machine_learning_server_amd.parallel.dist_miner import DistMiner
    tx = generate("ds2", seed=2)
    for mfma in (False, True):
        dm = DistMiner(tx.tx_ptr, tx.items, tx.n_items, 0.05, mfma=mfma, force_protocol=True)
        st = dm.step()["stats"]
        c = gpu_mod.mine_cpu(tx.tx_ptr, tx.items, tx.n_items, 0.05)
        assert st["global_itemsets"] == c["stats"]["n_itemsets"]


def test_default_arena_grows_on_demand(gpu_mod, monkeypatch):
    """A default-sized arena starts small (test hook arena_init_mb here; 8 GiB normally) and grows
    when the device-resident path runs out of room, instead of falling back or failing."""
    from kubernetes_machine_learning_server_amd.data.synthetic import generate
    monkeypatch.setenv("KMLS_TEST_HOOKS", "arena_init_mb=520")
    tx = generate("ds_dense", seed=3)
    g = gpu_mod.GpuMiner(0)
    assert g.arena_capacity < (600 << 20)
    g.load_csr(tx.tx_ptr, tx.items, tx.n_items)
    r = g.mine(0.05)
    assert r["stats"]["levels_path"] == "fused-resident", r["stats"]
    assert g.arena_capacity >= (2000 << 20)
    c = gpu_mod.mine_cpu(tx.tx_ptr, tx.items, tx.n_items, 0.05)
    assert r["stats"]["n_itemsets"] == c["stats"]["n_itemsets"]


@pytest.mark.parametrize("T,I", [(100_000, 1_000_000), (300_000, 1_012_345), (200_000, 40_000)])
def test_support_histograms_large_vocab(gpu_mod, T, I):
    """Both large-vocabulary support paths against np.bincount: the LDS-hash kernel (nnz < 4M)
    and the partitioned histogram (nnz >= 4M; vocabulary sizes not a multiple of 32768)."""
    import torch
    ptr, items = gpu_mod.synth_transactions(T, I, 30.0, 500, 0.9, 0.85, 7)
    g = gpu_mod.GpuMiner(0, 1 << 30, torch.cuda.current_stream().cuda_stream or 0)
    g.load_csr(ptr, items, I)
    cnt = torch.zeros(I, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    g.item_support(cnt.data_ptr())
    g.synchronize()
    np.testing.assert_array_equal(cnt.cpu().numpy().view(np.uint32),
                                  np.bincount(items, minlength=I))


def test_support_partitioned_count(gpu_mod):
    """The partitioned histogram (pass 3: equal global slices) on a Zipf-headed 1M vocabulary
    whose hot items repeat inside a thread's 8 ids, against np.bincount."""
    import torch
    ptr, items = gpu_mod.synth_transactions(400_000, 1_000_003, 30.0, 50, 0.95, 1.1, 11)
    g = gpu_mod.GpuMiner(0, 1 << 30, torch.cuda.current_stream().cuda_stream or 0)
    g.load_csr(ptr, items, 1_000_003)
    cnt = torch.zeros(1_000_003, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    g.item_support(cnt.data_ptr())
    g.synchronize()
    np.testing.assert_array_equal(cnt.cpu().numpy().view(np.uint32),
                                  np.bincount(items, minlength=1_000_003))


def test_graph_replay_matches_eager(gpu_mod):
    """Steady-state resident calls replay a captured hipGraph (third call on: the launch plan
    repeats); results must match the CPU miner on every call, including when the configuration
    alternates (key mismatch → recapture) and when results of earlier calls are still alive."""
    from kubernetes_machine_learning_server_amd.data.synthetic import generate
    tx = generate("ds2_weak", seed=6)
    ref = {ms: gpu_mod.mine_cpu(tx.tx_ptr, tx.items, tx.n_items, ms) for ms in (0.05, 0.04)}
    g = gpu_mod.GpuMiner(0, 1 << 31, 0)
    g.load_csr(tx.tx_ptr, tx.items, tx.n_items)
    kept, phases = [], []
    for ms in (0.05, 0.05, 0.05, 0.05, 0.04, 0.04, 0.04, 0.05, 0.05):
        r = g.mine(ms)
        assert r["stats"]["levels_path"] == "fused-resident", r["stats"]
        assert r["stats"]["n_itemsets"] == ref[ms]["stats"]["n_itemsets"]
        phases.append(next(k for k in r["stats"]["phases_ms"] if k.startswith("mine(graph")
                           or k.startswith("prologue")))
        kept.append((ms, r))
    assert "mine(graph replay)" in phases[2:4], phases
    for ms, r in kept:  # pinned results of replayed calls stay valid
        assert_same_itemsets(gpu_mod, r, ref[ms])
    small = [(ms, r) for ms, r in kept if r["stats"]["n_itemsets"] < 300_000][-1]
    assert _trie_dict(small[1]) == _trie_dict(ref[small[0]])


def test_prefetch_pipeline_matches_sync(gpu_mod):
    """mine(prefetch=True) launches the next identical call before waiting for the current one;
    the next mine() adopts it.  Every pipelined result (kept alive across later calls) must equal
    the CPU miner's, a configuration change must drop the launched-ahead call cleanly, and the
    partition entry point must pipeline the same way."""
    from kubernetes_machine_learning_server_amd.data.synthetic import generate
    tx = generate("ds2_weak", seed=7)
    ref = {ms: gpu_mod.mine_cpu(tx.tx_ptr, tx.items, tx.n_items, ms) for ms in (0.05, 0.04)}
    g = gpu_mod.GpuMiner(0, 1 << 31, 0)
    g.load_csr(tx.tx_ptr, tx.items, tx.n_items)
    kept, phases = [], []
    plan = [(0.05, False)] * 3 + [(0.05, True)] * 5 + [(0.05, False), (0.04, True), (0.04, True),
                                                      (0.05, True), (0.05, True), (0.05, False)]
    for ms, pre in plan:
        r = g.mine(ms, prefetch=pre)
        assert r["stats"]["n_itemsets"] == ref[ms]["stats"]["n_itemsets"], (ms, pre)
        phases.append(next(k for k in r["stats"]["phases_ms"] if k.startswith("mine(")))
        kept.append((ms, r))
    assert any("adopted" in p for p in phases), phases
    g.synchronize()
    for ms, r in kept:  # every result buffer stayed intact while later calls ran
        assert_same_itemsets(gpu_mod, r, ref[ms])
    assert _trie_dict(kept[6][1]) == _trie_dict(ref[0.05])
    # replicated-partition entry point: 2 ranks' pipelined sub-tries cover the full result
    total = 0
    for rank in (0, 1):
        h = gpu_mod.GpuMiner(0, 1 << 31, 0)
        h.load_csr(tx.tx_ptr, tx.items, tx.n_items)
        counts = []
        for i in range(6):
            r = h.mine_partition(0.05, 0, True, rank, 2, i < 5)
            counts.append(r["stats"]["n_itemsets"])
        assert len(set(counts)) == 1, counts
        total += counts[-1]
        del h
    assert total == ref[0.05]["stats"]["n_itemsets"]


@pytest.mark.parametrize("tiled", ["1", "0"])
def test_encode_long_shard_matches_onehot(gpu_mod, tiled, monkeypatch):
    """Bitmap encode of a long shard (>= 65536 transactions: the LDS-slab kernel, or the atomic
    kernel with the test hook encode_tiled=0) equals the one-hot matrix of the frequent items bit for bit,
    including a word offset into a wider buffer."""
    import torch
    from kubernetes_machine_learning_server_amd.data.synthetic import generate
    monkeypatch.setenv("KMLS_TEST_HOOKS", f"encode_tiled={tiled}")
    tx = generate("tiny", seed=12, n_tx=70001)
    g = gpu_mod.GpuMiner(0, 1 << 28, torch.cuda.current_stream().cuda_stream or 0)
    g.load_csr(tx.tx_ptr, tx.items, tx.n_items)
    cnt = torch.zeros(tx.n_items, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    g.item_support(cnt.data_ptr())
    g.synchronize()
    F = g.select(cnt.cpu().numpy().view(np.uint32), tx.n_tx, 0.02)
    ids, counts, _ = g.frequent()
    assert F > 4
    Wl = g.words_local()
    off = 3
    Wp = Wl + off + 1
    bm = torch.zeros((F, Wp), dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    g.encode_bitmaps(bm.data_ptr(), Wp, off)
    g.synchronize()
    words = bm.cpu().numpy().view(np.uint64)
    assert not words[:, :off].any() and not words[:, off + Wl:].any()
    bits = np.unpackbits(words[:, off:off + Wl].copy().view(np.uint8), axis=1,
                         bitorder="little")[:, :tx.n_tx]
    X = np.zeros((tx.n_tx, tx.n_items), dtype=np.uint8)
    for t in range(tx.n_tx):
        X[t, tx.items[tx.tx_ptr[t]:tx.tx_ptr[t + 1]]] = 1
    np.testing.assert_array_equal(bits, X[:, ids].T)


def _cpu_index(gpu_mod, tx, ms, names):
    from kubernetes_machine_learning_server_amd.serve.index import build_index_from_trie
    c = gpu_mod.mine_cpu(tx.tx_ptr, tx.items, tx.n_items, ms, 2)
    return build_index_from_trie(c["parent"], c["item"], c["count"], c["depth"], tx.n_tx,
                                 tx.n_items, names)


def _assert_index_equal(ix, ref, n_tx):
    np.testing.assert_array_equal(np.asarray(ix["row_ptr"]), ref.row_ptr)
    np.testing.assert_array_equal(np.asarray(ix["cons"]), ref.cons)
    np.testing.assert_array_equal(np.asarray(ix["count"], np.int64),
                                  np.rint(ref.score * n_tx).astype(np.int64))


@pytest.mark.parametrize("tie", ["names", "ids"])
@pytest.mark.parametrize("shape,ms,max_len", [("tiny", 0.05, 0), ("ds1", 0.05, 0),
                                              ("ds1", 0.01, 2), ("ds2_weak", 0.03, 0),
                                              ("ds_dense", 0.05, 0)])
def test_rule_index_on_device(gpu_mod, shape, ms, max_len, tie):
    """O10 pairs_to_csr: the rule map built from the resident gram == the CPU-built index
    (rows by item id, sorted by count desc then the tie key asc), and the mined trie is
    unaffected by building it."""
    from kubernetes_machine_learning_server_amd.data.synthetic import generate
    from kubernetes_machine_learning_server_amd.serve.index import name_tie_rank
    tx = generate(shape, seed=2)
    g = gpu_mod.GpuMiner(0)
    g.load_csr(tx.tx_ptr, tx.items, tx.n_items)
    names = tx.names if tie == "names" else None
    if names:
        g.set_tie_rank(name_tie_rank(names))
    ref = _cpu_index(gpu_mod, tx, ms, names)
    c = gpu_mod.mine_cpu(tx.tx_ptr, tx.items, tx.n_items, ms, max_len)
    # call 1 sizes the pinned host trie (full-width copy when it outgrows the first guess);
    # call 2 streams at compact widths, with the last level copied by the final copy-out
    for _ in range(2):
        r = g.mine(ms, max_len, rule_index=True)
        assert r["stats"]["levels_path"].startswith("fused"), r["stats"]
        _assert_index_equal(r["index"], ref, tx.n_tx)
        assert r["index"]["nnz"] == ref.nnz
        assert_same_itemsets(gpu_mod, r, c)


@pytest.mark.parametrize("shape,ms,n_tx,mfma", [("ds1", 0.05, None, True),
                                                ("ds2_weak", 0.02, 70000, False)])
def test_rule_map_from_gram(gpu_mod, shape, ms, n_tx, mfma):
    """The standalone device rule map (large-shape pipeline: caller-owned gram, banded encode
    into a stale buffer) == the CPU-built index; a too-small first capacity guess is redone at
    the exact size."""
    import torch
    from kubernetes_machine_learning_server_amd.data.synthetic import generate
    tx = generate(shape, seed=6, n_tx=n_tx)
    g = gpu_mod.GpuMiner(0, 1 << 28, torch.cuda.current_stream().cuda_stream or 0)
    g.load_csr(tx.tx_ptr, tx.items, tx.n_items)
    counts = np.bincount(tx.items, minlength=tx.n_items).astype(np.uint32)
    F = g.select(counts, tx.n_tx, ms)
    ids, fc, minsup = g.frequent()
    Wp = g.words_local()
    bm = torch.zeros((F, Wp), dtype=torch.int64, device="cuda")
    gram = torch.empty((F, F), dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    g.encode_bitmaps(bm.data_ptr(), Wp, 0)
    g.pair_counts(bm.data_ptr(), Wp, gram.data_ptr(), mfma)
    rm = g.rule_map_from_gram(gram.data_ptr(), F, int(minsup))
    assert rm["status"] == 0
    ref = _cpu_index(gpu_mod, tx, ms, None)
    _assert_index_equal(rm, ref, tx.n_tx)
    assert rm["nnz"] == ref.nnz


def test_rule_index_regrow_and_prefetch(gpu_mod, monkeypatch):
    """A too-small entry capacity regrows and redoes the call; launch-ahead calls adopt their
    own pinned CSR buffers (graph replay)."""
    monkeypatch.setenv("KMLS_TEST_HOOKS", "idx_cap=64")
    from kubernetes_machine_learning_server_amd.data.synthetic import generate
    from kubernetes_machine_learning_server_amd.serve.index import name_tie_rank
    tx = generate("ds1", seed=4)
    g = gpu_mod.GpuMiner(0)
    g.load_csr(tx.tx_ptr, tx.items, tx.n_items)
    g.set_tie_rank(name_tie_rank(tx.names))
    ref = _cpu_index(gpu_mod, tx, 0.05, tx.names)
    outs = [g.mine(0.05, rule_index=True, prefetch=(i < 4)) for i in range(5)]
    for r in outs:
        _assert_index_equal(r["index"], ref, tx.n_tx)


@pytest.mark.parametrize("fused", ["1", "0"])
def test_max_len_leaf_levels(gpu_mod, fused, monkeypatch):
    """Truncated mining (mlxtend max_len): the last allowed level is written as trie leaves
    without child bitmaps (chunked path) and must equal the CPU miner's truncated result."""
    from kubernetes_machine_learning_server_amd.data.synthetic import generate
    monkeypatch.setenv("KMLS_TEST_HOOKS", f"fused_levels={fused}")
    tx = generate("ds1", seed=6)
    g = gpu_mod.GpuMiner(0)
    g.load_csr(tx.tx_ptr, tx.items, tx.n_items)
    for ml in (3, 4):
        c = gpu_mod.mine_cpu(tx.tx_ptr, tx.items, tx.n_items, 0.02, ml)
        for _ in range(2):
            r = g.mine(0.02, ml)
            assert int(r["stats"]["max_depth"]) == ml
            assert_same_itemsets(gpu_mod, r, c)


@pytest.mark.parametrize("split", ["2", "3"])
def test_extend_split_k_long_rows(gpu_mod, monkeypatch, split):
    """Split-K extend (long rows sliced across teams, atomic partial counts, slice-0-only
    metadata): forced on a long-row chunked run, including an odd chunk remainder, and the trie
    must equal the CPU miner's."""
    from kubernetes_machine_learning_server_amd.data.synthetic import generate_large
    monkeypatch.setenv("KMLS_TEST_HOOKS", f"fused_levels=0,extend_split={split}")
    tx = generate_large("10Mx1M", seed=11, n_tx=300_000 + 64 * 7, n_items=50_000)
    before = gpu_mod.extend_split_launches()
    g = gpu_mod.GpuMiner(0)
    g.load_csr(tx.tx_ptr, tx.items, tx.n_items)
    r = g.mine(0.003)
    assert gpu_mod.extend_split_launches() > before, "the split path did not run"
    c = gpu_mod.mine_cpu(tx.tx_ptr, tx.items, tx.n_items, 0.003)
    assert int(c["stats"]["max_depth"]) >= 3
    assert_same_itemsets(gpu_mod, r, c)


@pytest.mark.parametrize("T,I,ms,min_f", [(300_000 + 37, 60_000, 0.002, 0),
                                            (200_000 + 37, 100_000, 0.002, 100),
                                            (300_000 + 37, 1_000_003, 0.001, 50),
                                            (200_000 + 37, 100_000, 0.0005, 3000)])
def test_encode_tiled_long_shard(gpu_mod, T, I, ms, min_f):
    """The LDS-slab encode produces the same tid-bitmaps as the host encoder, on a long shard
    with an odd tail tile; the second case has a million-style vocabulary (frequent-item mask
    in front of the rank gather, or the one-gather group tables when F <= 2048) and more
    frequent rows than one LDS slab (the multi-band kernel).  The buffer starts as all ones: the tiled encode must write every word of the shard's columns
    (the tx-DP path no longer clears the bitmap first)."""
    import torch
    ptr, items = gpu_mod.synth_transactions(T, I, 30.0, 500, 0.9, 0.85, 9)
    g = gpu_mod.GpuMiner(0, 1 << 30, torch.cuda.current_stream().cuda_stream or 0)
    g.load_csr(ptr, items, I)
    counts = np.bincount(items, minlength=I).astype(np.uint32)
    F = g.select(counts, T, ms)
    assert F >= min_f, F
    ids, fc, minsup = g.frequent()
    Wp = g.words_local()
    used = (T + 63) // 64
    bm = torch.full((F, Wp), -1, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    g.encode_bitmaps(bm.data_ptr(), Wp, 0)
    g.synchronize()
    sel = gpu_mod.select_frequent(counts, T, ms)
    ref = gpu_mod.encode_bitmaps_cpu(ptr, items, sel[2], F, Wp)
    np.testing.assert_array_equal(bm.cpu().numpy().view(np.uint64)[:, :used],
                                  ref.reshape(F, Wp)[:, :used])


def test_level_candidate_total_past_the_status_capacity(gpu_mod, monkeypatch):
    """64 transactions holding the same 1200 items: every itemset is frequent, and the level-3
    candidate total C(1200, 3) = 287,280,400 passes 2^28 (round 3's look-back limit).  With the
    look-back window shrunk (status_cap hook) past it, the capacity guard fires (overflow 4) and
    the chunked path produces the exact binomial counts; with the default window the level is
    counted (fused, or chunked when the device arena declines) with the same counts; the deep
    count-only miner agrees."""
    from math import comb
    T, I = 64, 1200
    tx_ptr = np.arange(T + 1, dtype=np.int64) * I
    items = np.tile(np.arange(I, dtype=np.int32), T)
    want = I + comb(I, 2) + comb(I, 3)
    monkeypatch.setenv("KMLS_TEST_HOOKS", "status_cap=65536")
    g = gpu_mod.GpuMiner(0)
    g.load_csr(tx_ptr, items, I)
    r = g.mine(0.5, 3, download=False)
    assert r["stats"]["n_itemsets"] == want
    assert "overflow code 4" in r["stats"].get("levels_path", "") or \
        "fallback" in r["stats"].get("levels_path", ""), r["stats"].get("levels_path")
    monkeypatch.delenv("KMLS_TEST_HOOKS")
    g2 = gpu_mod.GpuMiner(0)
    g2.load_csr(tx_ptr, items, I)
    r2 = g2.mine(0.5, 3, download=False)
    assert r2["stats"]["n_itemsets"] == want, r2["stats"].get("levels_path")
    d = g.mine_deep(0.5, 3)
    assert d["per_level"][1:4] == [I, comb(I, 2), comb(I, 3)]