"""Horizontal levels (csrc/kernels/hlevels.hip): sparse long transaction sets mined with no bitmap
at all — level 2 counted from the CSR (cooc.hip), levels >= 3 from a filtered CSR by hit lists
and candidate hash tables.  Every check is by content (trie digest: every (itemset, support)
pair) against the C++ CPU miner and against the bitmap levels of the same GPU miner; the trie
must list parents before children.  The reference mines every size (machine-learning/main.py:272)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _check_trie(par, dep):
    par = np.asarray(par, np.int64)
    idx = np.arange(len(par))
    assert (par < idx).all(), "a parent after its child"
    has = par >= 0
    dep = np.asarray(dep)
    assert (dep[has] == dep[par[has]] + 1).all()
    assert (dep[~has] == 1).all()


def _mine(gpu_mod, ptr, items, n_items, ms, max_len=0):
    g = gpu_mod.GpuMiner(0, 1 << 30, 0)
    g.load_csr(ptr, items, n_items)
    r = g.mine_txdp(None, len(ptr) - 1, ms, max_len)
    d = gpu_mod.trie_digest(r["parent"], r["item"], r["count"], r["depth"])
    return r, d


def _cpu(gpu_mod, ptr, items, n_items, ms, max_len=0):
    ref = gpu_mod.mine_cpu(ptr, items, n_items, ms, max_len)
    return gpu_mod.trie_digest(ref["parent"], ref["item"], ref["count"], ref["depth"])


def _long_rows(seed=0):
    """70k transactions (>= 1024 bitmap words) of sparse background noise, plus 2,000 that each
    hold 20 of 40 hot items: their filtered rows are longer than the 16-entry register sort."""
    rng = np.random.default_rng(seed)
    T, bg, hot = 70_000, 5000, 40
    rows = []
    for t in range(T):
        r = rng.choice(bg, 10, replace=False)
        if t % 35 == 0:
            r = np.concatenate([r, bg + rng.choice(hot, 20, replace=False)])
        rows.append(np.sort(r))
    ptr = np.zeros(T + 1, np.int64)
    ptr[1:] = np.cumsum([len(r) for r in rows])
    return ptr, np.concatenate(rows).astype(np.int32), bg + hot


@pytest.mark.parametrize("max_len", [0, 3])
def test_horizontal_levels_equal_cpu_and_bitmap_levels(gpu_mod, monkeypatch, max_len):
    T, I = 200_000, 50_000
    ptr, items = gpu_mod.synth_transactions(T, I, 25.0, 300, 0.9, 0.85, 9)
    ms = 1e-3
    monkeypatch.setenv("KMLS_TEST_HOOKS", "cooc=2")
    r, d = _mine(gpu_mod, ptr, items, I, ms, max_len)
    st = r["stats"]
    assert st["levels_path"] == "horizontal" and "encode_bitmap" not in st["phases_ms"]
    h = st["horizontal"]
    assert h["tx_kept"] > 0
    if max_len == 0:
        assert len(h["per_level"]) >= 2  # sizes 2 and 3 at least
    _check_trie(r["parent"], r["depth"])
    monkeypatch.setenv("KMLS_TEST_HOOKS", "cooc=2,hlevels=0")
    rb, db = _mine(gpu_mod, ptr, items, I, ms, max_len)
    assert rb["stats"]["levels_path"] != "horizontal"
    want = _cpu(gpu_mod, ptr, items, I, ms, max_len)
    assert d["digest"] == db["digest"] == want["digest"]
    assert d["per_depth"] == want["per_depth"]
    if max_len:
        assert max(np.asarray(r["depth"])) <= max_len


def test_horizontal_long_rows_and_regrown_buffers(gpu_mod, monkeypatch):
    """Filtered rows of 20 items (in-place sort path) and every buffer started tiny (hl_cap:
    the filter and the hit passes re-run with the exact sizes their counters reached)."""
    ptr, items, n_items = _long_rows()
    ms = 200 / 70_000
    want = _cpu(gpu_mod, ptr, items, n_items, ms)
    assert want["per_depth"][3] > 0  # triples of hot items are frequent
    for hooks in ("cooc=2", "cooc=2,hl_cap=64", "cooc=2,pair_rows=0"):
        monkeypatch.setenv("KMLS_TEST_HOOKS", hooks)
        r, d = _mine(gpu_mod, ptr, items, n_items, ms)
        assert r["stats"]["levels_path"] == "horizontal"
        assert d["digest"] == want["digest"], hooks
        _check_trie(r["parent"], r["depth"])


def test_horizontal_pairs_only_and_empty(gpu_mod, monkeypatch):
    """max_len 2 stops after the pair table; a support with no frequent pair gives level 1 only."""
    ptr, items, n_items = _long_rows(seed=1)
    monkeypatch.setenv("KMLS_TEST_HOOKS", "cooc=2")
    for ms, ml in ((200 / 70_000, 2), (0.5, 0)):
        r, d = _mine(gpu_mod, ptr, items, n_items, ms, ml)
        assert d["digest"] == _cpu(gpu_mod, ptr, items, n_items, ms, ml)["digest"]


def _wide_vocab(seed=0):
    """60k frequent items, so most ranks are past 32768: 45k 'head' items in ~60 transactions
    each, 15k 'tail' items in ~30; 1,500 tail pairs planted in 25 transactions each and 100 tail
    triples in 25 each — their items then hold ~55 transactions, ranks 45,000 and up.  300k
    transactions (>= 1024 bitmap words: the horizontal path's long-shard rule)."""
    rng = np.random.default_rng(seed)
    T, H, Tl = 300_000, 45_000, 15_000
    I = H + Tl
    it = [np.repeat(np.arange(H), 60), np.repeat(H + np.arange(Tl), 30)]
    tx = [rng.integers(0, T, H * 60), rng.integers(0, T, Tl * 30)]
    tail = H + rng.permutation(Tl)
    pairs = tail[:3000].reshape(-1, 2)
    triples = tail[3000:3300].reshape(-1, 3)
    for sets in (pairs, triples):
        for s in sets:
            t = rng.choice(T, 25, replace=False)
            for x in s:
                it.append(np.full(25, x))
                tx.append(t)
    key = np.unique(np.concatenate(tx).astype(np.int64) * I + np.concatenate(it))
    txs, items = key // I, (key % I).astype(np.int32)
    ptr = np.zeros(T + 1, np.int64)
    np.add.at(ptr, txs + 1, 1)
    return np.cumsum(ptr), items, I


def _reference_trie(ptr, items, I, minc):
    """Every frequent itemset of the wide-vocabulary data, computed without a miner: supports by
    bincount, pairs from the sparse co-occurrence X^T X, triples (and up) by intersecting the
    transaction sets of candidates whose every sub-itemset is frequent."""
    import scipy.sparse as sp
    T = len(ptr) - 1
    X = sp.csr_matrix((np.ones(len(items), np.int32), items, ptr), shape=(T, I))
    sup = np.bincount(items, minlength=I)
    freq = {(int(i),): int(sup[i]) for i in np.nonzero(sup >= minc)[0]}
    C = sp.triu(X.T @ X, k=1).tocoo()
    keep = C.data >= minc
    level = {(int(a), int(b)): int(c) for a, b, c in zip(C.row[keep], C.col[keep], C.data[keep])}
    freq.update(level)
    Xc = X.tocsc()
    tids = {}

    def tid(i):
        if i not in tids:
            tids[i] = set(Xc.indices[Xc.indptr[i]:Xc.indptr[i + 1]].tolist())
        return tids[i]
    while level:
        keys = sorted(level)
        nxt = {}
        for x in range(len(keys)):
            for y in range(x + 1, len(keys)):
                a, b = keys[x], keys[y]
                if a[:-1] != b[:-1]:
                    break
                cand = a + (b[-1],)
                if all(tuple(cand[:k] + cand[k + 1:]) in level for k in range(len(cand))):
                    s = set.intersection(*(tid(i) for i in cand))
                    if len(s) >= minc:
                        nxt[cand] = len(s)
        freq.update(nxt)
        level = nxt
    node, parent, item, count, depth = {}, [], [], [], []
    for s in sorted(freq, key=len):
        node[s] = len(parent)
        parent.append(node[s[:-1]] if len(s) > 1 else -1)
        item.append(s[-1])
        count.append(freq[s])
        depth.append(len(s))
    return (np.asarray(parent, np.int64), np.asarray(item, np.int32),
            np.asarray(count, np.uint32), np.asarray(depth, np.uint8))


def test_horizontal_levels_past_32768_ranks(gpu_mod, monkeypatch):
    """The sparse path with 60k frequent items (16-bit ranks up to 65,534, 0xFFFF = none): pair
    rows and horizontal levels over ranks > 32768, digest-equal to an independent reference
    (scipy co-occurrence + transaction-set intersections; mine_cpu's F x F bitmap pairs are out
    of reach at this F)."""
    ptr, items, I = _wide_vocab()
    T = len(ptr) - 1
    minc = 20
    ms = (minc - 0.5) / T
    assert gpu_mod.level1_threshold(T, ms) == minc
    want = gpu_mod.trie_digest(*_reference_trie(ptr, items, I, minc))
    assert want["per_depth"][1] > 40_000 and want["per_depth"][2] >= 1500
    assert want["per_depth"][3] >= 100
    monkeypatch.setenv("KMLS_TEST_HOOKS", "cooc=2")
    g = gpu_mod.GpuMiner(0, 0, 0)  # auto arena: the dense 60k x 60k level-2 gram is 14.4 GB
    g.load_csr(ptr, items, I)
    r = g.mine_txdp(None, T, ms, 0)
    assert r["stats"]["levels_path"] == "horizontal"
    assert r["stats"]["n_frequent_items"] > 40_000
    d = gpu_mod.trie_digest(r["parent"], r["item"], r["count"], r["depth"])
    assert d["per_depth"] == want["per_depth"]
    assert d["digest"] == want["digest"]
    _check_trie(r["parent"], r["depth"])
