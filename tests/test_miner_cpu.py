"""CPU parity tests: oracle (mlxtend-faithful FP-tree) vs brute force vs the native C++ miner.

SURVEY §7.6: hand-computed tiny cases, encoder dedup, the ``ms*T`` threshold edge, single-path
combinatorics, and the rule-map == pair-support property.
"""
import math

import numpy as np
import pytest
from hypothesis import given, settings, strategies as st

from kubernetes_machine_learning_server_amd.data.synthetic import generate
from kubernetes_machine_learning_server_amd.models import oracle
from kubernetes_machine_learning_server_amd.models.fpgrowth import (TransactionEncoder, fpgrowth,
                                                                    mine_csr)


def trie_sets(trie):
    return {frozenset(s): c for c, s in trie.itemsets()}


def test_hand_computed_tiny():
    tx = [["a", "b", "c"], ["a", "b"], ["a", "c"], ["b", "c"], ["a", "b", "c", "a"]]
    X, cols = oracle.transaction_encode(tx)
    assert cols == ["a", "b", "c"]
    assert X.sum() == 12  # duplicate "a" collapsed
    res = {s: round(sup * 5) for sup, s in oracle.fpgrowth_oracle(X, 0.4, cols)}
    assert res == {frozenset("a"): 4, frozenset("b"): 4, frozenset("c"): 4,
                   frozenset("ab"): 3, frozenset("ac"): 3, frozenset("bc"): 3,
                   frozenset("abc"): 2}
    # the same through every backend of the public API
    for backend in ("oracle", "cpu"):
        df = fpgrowth(__import__("pandas").DataFrame(X, columns=cols), 0.4, use_colnames=True,
                      backend=backend)
        got = {s: round(sup * 5) for sup, s in zip(df["support"], df["itemsets"])}
        assert got == res


def test_threshold_float_quirk():
    """level 1 uses count/T >= ms, deeper levels ceil(ms*T): 0.07*100 = 7.000000000000001."""
    assert math.ceil(0.07 * 100) == 8
    assert oracle.level1_is_frequent(7, 100, 0.07)
    assert oracle.level2_threshold(100, 0.07) == 8
    # 7 transactions contain {x, y}; 93 contain {z}
    tx = [["x", "y"]] * 7 + [["z"]] * 93
    X, cols = oracle.transaction_encode(tx)
    o = {s: c for c, s in ((round(s * 100), it) for s, it in oracle.fpgrowth_oracle(X, 0.07, cols))}
    # x, y are frequent singles, the pair {x,y} (count 7 < 8) is not ... unless the root tree is
    # a single path (it is not here: z is a separate branch)
    assert frozenset(["x"]) in o and frozenset(["y"]) in o and frozenset(["x", "y"]) not in o
    ptr = np.array([0] + list(np.cumsum([2] * 7 + [1] * 93)), dtype=np.int64)
    items = np.array([0, 1] * 7 + [2] * 93, dtype=np.int32)
    t = mine_csr(ptr, items, 3, 0.07, backend="cpu")
    assert trie_sets(t) == {frozenset([0]): 7, frozenset([1]): 7, frozenset([2]): 93}


def test_single_path_combinations():
    tx = [["a", "b", "c"]] * 4 + [["a", "b"]] * 2 + [["a"]]
    X, cols = oracle.transaction_encode(tx)
    o = {s: round(sup * 7) for sup, s in oracle.fpgrowth_oracle(X, 0.2, cols)}
    b = oracle.frequent_itemsets_bruteforce(X, 0.2)
    assert o == {frozenset(cols[i] for i in s): c for s, c in b.items()}
    assert o[frozenset("abc")] == 4


@pytest.mark.parametrize("shape,ms", [("tiny", 0.05), ("tiny", 0.1), ("tiny", 0.02)])
def test_cpu_miner_vs_oracle_and_bruteforce(shape, ms):
    tx = generate(shape, seed=1)
    X = tx.onehot()
    o = {frozenset(s): round(sup * tx.n_tx) for sup, s in oracle.fpgrowth_oracle(X, ms)}
    b = oracle.frequent_itemsets_bruteforce(X, ms)
    c = trie_sets(mine_csr(tx.tx_ptr, tx.items, tx.n_items, ms, backend="cpu"))
    assert o == b == c


@settings(max_examples=40, deadline=None)
@given(st.integers(1, 60), st.integers(1, 12), st.floats(0.05, 0.6), st.integers(0, 2**31 - 1))
def test_cpu_miner_property(n_tx, n_items, ms, seed):
    rng = np.random.default_rng(seed)
    dens = rng.uniform(0.1, 0.8)
    X = rng.random((n_tx, n_items)) < dens
    rows, cols = np.nonzero(X)
    ptr = np.zeros(n_tx + 1, np.int64)
    np.add.at(ptr, rows + 1, 1)
    ptr = np.cumsum(ptr)
    b = oracle.frequent_itemsets_bruteforce(X, ms)
    c = trie_sets(mine_csr(ptr, cols.astype(np.int32), n_items, ms, backend="cpu"))
    o = {frozenset(s): round(sup * n_tx) for sup, s in oracle.fpgrowth_oracle(X, ms)}
    assert c == b
    assert o == b


@pytest.mark.parametrize("max_len", [1, 2, 3])
def test_max_len(max_len):
    tx = generate("tiny", seed=4)
    X = tx.onehot()
    o = {frozenset(s): round(sup * tx.n_tx)
         for sup, s in oracle.fpgrowth_oracle(X, 0.02, max_len=max_len)}
    c = trie_sets(mine_csr(tx.tx_ptr, tx.items, tx.n_items, 0.02, max_len=max_len, backend="cpu"))
    assert o == c
    assert max(len(s) for s in c) <= max_len


def test_rule_map_equals_pair_support():
    """the reference rule map depends only on frequent 1- and 2-itemsets."""
    tx = generate("tiny", seed=7)
    X = tx.onehot()
    for ms in (0.1, 0.05, 0.02):
        recs = oracle.fpgrowth_oracle(X, ms)
        full = oracle.rule_map_from_itemsets(recs)
        singles = [(next(iter(s)), sup) for sup, s in recs if len(s) == 1]
        pairs = [tuple(sorted(s)) + (sup,) for sup, s in recs if len(s) == 2]
        short = oracle.rule_map_from_pairs(singles, pairs)
        assert full == short


def test_transaction_encoder_api():
    te = TransactionEncoder()
    tx = [["b", "a"], ["c"], ["a", "a", "c"]]
    X = te.fit(tx).transform(tx)
    assert te.columns_ == ["a", "b", "c"]
    assert X.tolist() == [[True, True, False], [False, False, True], [True, False, True]]
    ptr, items = te.to_csr(tx)
    assert ptr.tolist() == [0, 2, 3, 5] and items.tolist() == [0, 1, 2, 0, 2]


def test_fpgrowth_rejects_bad_input():
    with pytest.raises(ValueError):
        fpgrowth(np.array([[0, 2]]), 0.5)
    with pytest.raises(ValueError):
        mine_csr(np.array([0, 1]), np.array([0], np.int32), 1, 0.0)


def test_ds2_shape_calibration():
    """Synthetic ds2 reproduces the published shape (relatorio.pdf p.5-6)."""
    from kubernetes_machine_learning_server_amd.data.synthetic import item_support_curve
    tx = generate("ds2", seed=0)
    assert tx.n_tx == 2246 and tx.n_items == 2171
    assert abs(len(tx.items) - 240249 / 1.01) / 240249 < 0.03
    curve = dict(item_support_curve(tx, [0.03, 0.05, 0.1]))
    assert abs(curve[0.05] - 755) < 80 and abs(curve[0.03] - 1571) < 120
    assert abs(curve[0.1] - 121) < 30


@pytest.mark.parametrize("ms,max_len", [(0.05, 0), (0.04, 0), (0.04, 3), (0.05, 2)])
def test_count_digest_equals_trie_digest(native_mod, ms, max_len):
    """mine_cpu_count's digest (no trie) is the digest of the full CPU trie."""
    from kubernetes_machine_learning_server_amd.data.synthetic import generate
    tx = generate("ds1", seed=0)
    c = native_mod.mine_cpu_count(tx.tx_ptr, tx.items, tx.n_items, ms, max_len)
    r = native_mod.mine_cpu(tx.tx_ptr, tx.items, tx.n_items, ms, max_len)
    d = native_mod.trie_digest(r["parent"], r["item"], r["count"], r["depth"])
    assert c["digest"] == d["digest"]
    assert c["per_level"][1:] == d["per_depth"][1:]
    assert c["n_itemsets"] == d["n"]
