"""Association rules over a mined :class:`ItemsetTrie`.

* :func:`association_rules` — the ``mlxtend.frequent_patterns.association_rules`` surface
  (antecedent/consequent support, support, confidence, lift, leverage, conviction,
  zhangs_metric, jaccard, certainty, kulczynski) computed by the native rule engine
  (``csrc/host/rules_cpu.cpp``: every antecedent subset of every frequent itemset, supports
  looked up in the trie).
* :func:`fpgrowth_py` — ``fpgrowth_py.fpgrowth(transactions, minSupRatio, minConf)``
  semantics of the reference's legacy path (``machine-learning/main.py:224-260``): frequent
  itemsets with ``count >= T * minSupRatio`` and rules ``[set(A), set(C), conf]`` with
  ``conf > minConf`` (strict).  Returns ``None`` when nothing is frequent, as the library.
* :func:`confidence_rule_map` — what the legacy path MEANT to build (it crashes on unhashable
  set keys): ``song -> {other: max confidence}`` from single-song
  antecedents; usable as an alternative recommendations map (``RULES_METRIC=confidence``).
"""
from __future__ import annotations

from typing import Dict, Hashable, Iterable, List, Optional, Sequence

import numpy as np

from ..ops import native
from .fpgrowth import ItemsetTrie, csr_from_lists, mine_csr

_METRICS = {"confidence": 0, "lift": 1, "leverage": 2, "support": 3, "conviction": 4}


class Rules:
    """Columnar rule set: trie node ids of (itemset, antecedent, consequent) + metrics."""

    def __init__(self, trie: ItemsetTrie, raw: Dict[str, np.ndarray]):
        self.trie = trie
        self.itemset = np.asarray(raw["itemset"])
        self.antecedent = np.asarray(raw["antecedent"])
        self.consequent = np.asarray(raw["consequent"])
        self.confidence = np.asarray(raw["confidence"])
        self.lift = np.asarray(raw["lift"])

    def __len__(self) -> int:
        return len(self.itemset)

    def _sets(self, nodes: np.ndarray, use_colnames: bool) -> List[frozenset]:
        t = self.trie
        cols = t.columns if (use_colnames and t.columns is not None) else None
        cache: Dict[int, frozenset] = {}

        def items(v: int) -> frozenset:
            if v in cache:
                return cache[v]
            out = []
            u = v
            while u >= 0:
                out.append(int(t.item[u]))
                u = int(t.parent[u])
            fs = frozenset(cols[i] for i in out) if cols is not None else frozenset(out)
            cache[v] = fs
            return fs
        return [items(int(v)) for v in nodes]

    def to_dataframe(self, use_colnames: bool = True):
        import pandas as pd
        t = self.trie
        T = float(t.n_tx)
        sS = t.count[self.itemset] / T
        sA = t.count[self.antecedent] / T
        sC = t.count[self.consequent] / T
        conf = self.confidence
        with np.errstate(divide="ignore", invalid="ignore"):
            lev = sS - sA * sC
            conv = np.where(conf >= 1.0, np.inf, (1.0 - sC) / (1.0 - conf))
            denom = np.maximum(sS * (1 - sA), sA * (sC - sS))
            zhang = np.where(denom == 0, 0.0, lev / np.where(denom == 0, 1.0, denom))
            jacc = sS / (sA + sC - sS)
            cert = np.where(sC >= 1.0, 0.0, (conf - sC) / (1.0 - sC))
            kulc = 0.5 * (sS / sA + sS / sC)
        return pd.DataFrame({
            "antecedents": self._sets(self.antecedent, use_colnames),
            "consequents": self._sets(self.consequent, use_colnames),
            "antecedent support": sA, "consequent support": sC, "support": sS,
            "confidence": conf, "lift": self.lift, "representativity": np.ones(len(self)),
            "leverage": lev, "conviction": conv, "zhangs_metric": zhang, "jaccard": jacc,
            "certainty": cert, "kulczynski": kulc,
        })


def rules_from_trie(trie: ItemsetTrie, metric: str = "confidence", min_threshold: float = 0.8,
                    max_antecedent: int = 0, strict: bool = False, backend: str = "auto",
                    device: int = 0) -> Rules:
    """``backend``: "gpu" (HIP rule_score kernels, csrc/kernels/rules.hip), "cpu" (threaded
    C++), "auto" (GPU when one is visible and the trie is large enough to amortise the upload).
    Both produce identical rules in identical order."""
    if metric not in _METRICS:
        raise ValueError(f"unknown metric {metric!r}; choose from {sorted(_METRICS)}")
    m = 5 if (strict and metric == "confidence") else _METRICS[metric]
    args = (np.ascontiguousarray(trie.parent, np.int64), np.ascontiguousarray(trie.item, np.int32),
            np.ascontiguousarray(trie.count, np.uint32), np.ascontiguousarray(trie.depth, np.uint8),
            int(trie.n_tx), m, float(min_threshold), int(max_antecedent))
    if backend == "auto":
        backend = "gpu" if (len(trie) >= 50_000 and native.gpu_available()) else "cpu"
    if backend == "gpu":
        raw = native.require_gpu().association_rules_gpu(*args, device)
    elif backend == "cpu":
        raw = native.load().association_rules(*args)
    else:
        raise ValueError(f"unknown backend {backend!r}")
    return Rules(trie, raw)


def association_rules(frequent, num_itemsets: Optional[int] = None, metric: str = "confidence",
                      min_threshold: float = 0.8, support_only: bool = False,
                      use_colnames: bool = True):
    """mlxtend-compatible entry point.  ``frequent`` is an :class:`ItemsetTrie` (as returned by
    ``fpgrowth(..., as_trie=True)``) — the DataFrame form is accepted too (re-indexed)."""
    trie = frequent if isinstance(frequent, ItemsetTrie) else _trie_from_df(frequent, num_itemsets)
    if support_only:
        metric, min_threshold = "support", 0.0
    return rules_from_trie(trie, metric, min_threshold).to_dataframe(use_colnames)


def _trie_from_df(df, num_itemsets: Optional[int]) -> ItemsetTrie:
    if num_itemsets is None:
        raise ValueError("num_itemsets (the transaction count) is required for a DataFrame input")
    from .fpgrowth import _trie_from_records
    cols = sorted({it for s in df["itemsets"] for it in s}, key=repr)
    cid = {c: i for i, c in enumerate(cols)}
    recs = [(sup, frozenset(cid[i] for i in s)) for sup, s in zip(df["support"], df["itemsets"])]
    t = _trie_from_records(recs, int(num_itemsets), float(min(df["support"], default=0.0)), cols)
    return _reorder_for_lookup(t)


def _reorder_for_lookup(t: ItemsetTrie) -> ItemsetTrie:
    """_trie_from_records builds paths in ascending item-id order, which is a valid global order
    for subset lookup (every path increasing) — nothing to do."""
    return t


def fpgrowth_py(transactions: Sequence[Iterable[Hashable]], minSupRatio: float = 0.5,
                minConf: float = 0.5, backend: str = "auto"):
    """``fpgrowth_py.fpgrowth`` (reference legacy path): ``(freqItemSet, rules)`` or ``None``."""
    tx = [list(t) for t in transactions]
    vocab = sorted({it for t in tx for it in t}, key=repr)
    mapping = {c: i for i, c in enumerate(vocab)}
    ptr, items = csr_from_lists(tx, mapping)
    trie = mine_csr(ptr, items, len(vocab), minSupRatio, backend=backend, columns=vocab)
    if len(trie) == 0:
        return None
    freq = [set(s) for _, s in trie.to_records(True)]
    r = rules_from_trie(trie, "confidence", minConf, strict=True)
    A = r._sets(r.antecedent, True)
    C = r._sets(r.consequent, True)
    rules = [[set(a), set(c), float(conf)] for a, c, conf in zip(A, C, r.confidence)]
    return freq, rules


def confidence_rule_map(rules, singles: Iterable[Hashable] = ()) -> Dict:
    """``song -> {other: max confidence}`` over rules with a single-song antecedent (what
    ``calculate_and_save_fp_growth`` intended, main.py:240-250).  Every frequent single song
    is a key (possibly with ``{}``), mirroring the deployed map's key set."""
    rec: Dict = {s: {} for s in singles}
    for ante, cons, conf in rules:
        if len(ante) != 1:
            continue
        (a,) = tuple(ante)
        row = rec.setdefault(a, {})
        for c in cons:
            prev = row.get(c)
            row[c] = conf if prev is None else max(prev, conf)
    return rec
