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
