"""Association rules vs brute force over oracle itemsets; fpgrowth_py compat."""
import itertools

import numpy as np
import pytest

from kubernetes_machine_learning_server_amd.data.synthetic import generate
from kubernetes_machine_learning_server_amd.models import oracle
from kubernetes_machine_learning_server_amd.models.fpgrowth import fpgrowth, mine_csr
from kubernetes_machine_learning_server_amd.models.rules import (association_rules,
                                                                 confidence_rule_map, fpgrowth_py,
                                                                 rules_from_trie)


def brute_rules(freq, T, metric, thr, strict=False):
    out = {}
    for S, cS in freq.items():
        if len(S) < 2:
            continue
        for r in range(1, len(S)):
            for A in itertools.combinations(sorted(S), r):
                A = frozenset(A)
                C = S - A
                conf = cS / freq[A]
                lift = conf / (freq[C] / T)
                lev = cS / T - (freq[A] / T) * (freq[C] / T)
                val = {"confidence": conf, "lift": lift, "leverage": lev}[metric]
                if (val > thr) if strict else (val >= thr - 1e-12):
                    out[(A, C)] = (conf, lift)
    return out


@pytest.mark.parametrize("ms,metric,thr", [(0.05, "confidence", 0.3), (0.03, "confidence", 0.6),
                                           (0.05, "lift", 1.5), (0.05, "leverage", 0.005)])
def test_rules_match_bruteforce(ms, metric, thr):
    tx = generate("tiny", seed=2)
    trie = mine_csr(tx.tx_ptr, tx.items, tx.n_items, ms, backend="cpu")
    freq = {frozenset(s): c for c, s in trie.itemsets()}
    ref = brute_rules(freq, tx.n_tx, metric, thr)
    r = rules_from_trie(trie, metric, thr)
    A, C = r._sets(r.antecedent, False), r._sets(r.consequent, False)
    got = {(a, c): (cf, lf) for a, c, cf, lf in zip(A, C, r.confidence, r.lift)}
    assert set(got) == set(ref)
    for k in ref:
        assert np.isclose(got[k][0], ref[k][0]) and np.isclose(got[k][1], ref[k][1])


def test_association_rules_dataframe_shape():
    tx = generate("tiny", seed=3)
    lists = tx.to_lists()
    X, cols = oracle.transaction_encode(lists)
    import pandas as pd
    trie = fpgrowth(pd.DataFrame(X, columns=cols), 0.05, use_colnames=True, backend="cpu",
                    as_trie=True)
    df = association_rules(trie, metric="confidence", min_threshold=0.5)
    assert list(df.columns[:7]) == ["antecedents", "consequents", "antecedent support",
                                    "consequent support", "support", "confidence", "lift"]
    assert (df["confidence"] >= 0.5).all()
    row = df.iloc[0]
    assert np.isclose(row["confidence"], row["support"] / row["antecedent support"])
    assert np.isclose(row["lift"], row["confidence"] / row["consequent support"])
    # DataFrame input (mlxtend style) gives the same rules
    fi = trie.to_dataframe(True)
    df2 = association_rules(fi, num_itemsets=tx.n_tx, metric="confidence", min_threshold=0.5)
    key = lambda d: sorted((tuple(sorted(a)), tuple(sorted(c)), round(x, 9))
                           for a, c, x in zip(d["antecedents"], d["consequents"], d["confidence"]))
    assert key(df) == key(df2)


def test_fpgrowth_py_compat_matches_oracle():
    tx = generate("tiny", seed=5)
    lists = [[f"s{i}" for i in r] for r in tx.to_lists()]
    freq, rules = fpgrowth_py(lists, 0.05, 0.4, backend="cpu")
    ofreq, orules = oracle.fpgrowth_py_rules_oracle(lists, 0.05, 0.4)
    assert sorted(map(sorted, freq)) == sorted(map(sorted, ofreq))
    k = lambda rs: sorted((tuple(sorted(a)), tuple(sorted(c)), round(x, 12)) for a, c, x in rs)
    assert k(rules) == k(orules)
    assert all(x > 0.4 for _, _, x in rules)  # strict
    assert fpgrowth_py([["a"], ["b"]], 0.9, 0.1, backend="cpu") is None
    rec = confidence_rule_map(rules, singles=[next(iter(s)) for s in freq if len(s) == 1])
    for ante, cons, conf in rules:
        if len(ante) == 1:
            (a,) = tuple(ante)
            for c in cons:
                assert rec[a][c] >= conf
