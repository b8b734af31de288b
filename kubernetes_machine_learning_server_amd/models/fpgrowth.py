"""Public FP-Growth API (mlxtend-compatible surface) over the native CPU / HIP miners.

``fpgrowth(df, min_support, use_colnames, max_len)`` mirrors
``mlxtend.frequent_patterns.fpgrowth`` as called by the reference
(``machine-learning/main.py:272``), and ``TransactionEncoder`` mirrors
``mlxtend.preprocessing.TransactionEncoder`` (``main.py:267-269``).  Results are produced as an
:class:`ItemsetTrie` — the compact form every miner emits (node = parent itemset + one item,
with its support count) — and materialised to the mlxtend DataFrame only on request.

Backends: ``"gpu"`` (HIP kernels: the deep DFS miner, csrc/kernels/deep.hip, for short
transaction sets; the level-wise miner, csrc/kernels/levels.hip, otherwise), ``"cpu"`` (C++ bitmap Eclat,
csrc/host/miner_cpu.cpp), ``"oracle"`` (pure-Python mlxtend-faithful FP-tree, models/oracle.py).
``"auto"`` = gpu if a HIP device is visible, else cpu.
"""
from __future__ import annotations

import dataclasses
import os
from typing import Dict, Hashable, Iterable, Iterator, List, Optional, Sequence, Tuple

import numpy as np

from ..ops import native
from . import oracle as _oracle

__all__ = ["TransactionEncoder", "ItemsetTrie", "fpgrowth", "mine_csr", "csr_from_lists",
           "default_backend", "full_miner"]


# --------------------------------------------------------------------------------------------
class TransactionEncoder:
    """``mlxtend.preprocessing.TransactionEncoder``: columns_ = sorted unique items."""

    def fit(self, X: Sequence[Iterable[Hashable]]) -> "TransactionEncoder":
        self.columns_ = sorted({it for tx in X for it in tx})
        self.columns_mapping_ = {c: i for i, c in enumerate(self.columns_)}
        return self

    def transform(self, X: Sequence[Iterable[Hashable]], sparse: bool = False) -> np.ndarray:
        out = np.zeros((len(X), len(self.columns_)), dtype=bool)
        m = self.columns_mapping_
        for r, tx in enumerate(X):
            idx = [m[it] for it in tx]
            out[r, idx] = True
        return out

    def fit_transform(self, X, sparse: bool = False):
        return self.fit(X).transform(X, sparse=sparse)

    def to_csr(self, X: Sequence[Iterable[Hashable]]) -> Tuple[np.ndarray, np.ndarray]:
        """CSR form (what the miners consume) without the dense T x I matrix."""
        return csr_from_lists(X, self.columns_mapping_)


def csr_from_lists(X: Sequence[Iterable[Hashable]], mapping: Dict[Hashable, int]
                   ) -> Tuple[np.ndarray, np.ndarray]:
    ptr = np.zeros(len(X) + 1, dtype=np.int64)
    rows = []
    for r, tx in enumerate(X):
        row = np.unique(np.fromiter((mapping[it] for it in tx), dtype=np.int32))
        rows.append(row)
        ptr[r + 1] = ptr[r] + len(row)
    items = np.concatenate(rows) if rows else np.zeros(0, np.int32)
    return ptr, items.astype(np.int32)


# --------------------------------------------------------------------------------------------
@dataclasses.dataclass
class ItemsetTrie:
    """All frequent itemsets: node n = itemset(parent[n]) ∪ {item[n]} with support count[n]."""
    parent: np.ndarray
    item: np.ndarray
    count: np.ndarray
    depth: np.ndarray
    n_tx: int
    min_support: float
    stats: Dict = dataclasses.field(default_factory=dict)
    columns: Optional[Sequence] = None

    def __len__(self) -> int:
        return int(len(self.item))

    @property
    def support(self) -> np.ndarray:
        return self.count / float(self.n_tx)

    def itemsets(self) -> Iterator[Tuple[int, Tuple[int, ...]]]:
        """(count, itemset as tuple of item ids) for every node, trie order."""
        memo: List[Tuple[int, ...]] = []
        for n in range(len(self.item)):
            p = int(self.parent[n])
            s = (memo[p] if p >= 0 else ()) + (int(self.item[n]),)
            memo.append(s)
            yield int(self.count[n]), s

    def as_dict(self) -> Dict[frozenset, int]:
        return {frozenset(s): c for c, s in self.itemsets()}

    def to_records(self, use_colnames: bool = True) -> List[Tuple[float, frozenset]]:
        cols = self.columns
        out = []
        for c, s in self.itemsets():
            names = [cols[i] for i in s] if (use_colnames and cols is not None) else list(s)
            out.append((c / self.n_tx, frozenset(names)))
        return out

    def to_dataframe(self, use_colnames: bool = True):
        """mlxtend's result: DataFrame[support: float, itemsets: frozenset]."""
        import pandas as pd
        recs = self.to_records(use_colnames)
        return pd.DataFrame({"support": [r[0] for r in recs], "itemsets": [r[1] for r in recs]})

    def singles(self) -> Tuple[np.ndarray, np.ndarray]:
        m = self.depth == 1
        return self.item[m], self.count[m]

    def pairs(self) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        """Frequent 2-itemsets (a, b, count); a = parent item."""
        m = self.depth == 2
        par = self.parent[m]
        return self.item[par], self.item[m], self.count[m]

    def size_histogram(self) -> Dict[int, int]:
        h = np.bincount(self.depth.astype(np.int64))
        return {int(k): int(v) for k, v in enumerate(h) if v}


# --------------------------------------------------------------------------------------------
def default_backend() -> str:
    env = os.environ.get("MINER", "").lower()
    if env in ("gpu", "cpu", "oracle"):
        return env
    return "gpu" if native.gpu_available() else "cpu"


_GPU_MINER = None


def _gpu_miner():
    global _GPU_MINER
    if _GPU_MINER is None:
        m = native.require_gpu()
        _GPU_MINER = m.GpuMiner(int(os.environ.get("KMLS_DEVICE", "0")))
    return _GPU_MINER


DEEP_MAX_TX = 4096  # the deep miner's tid rows: at most 64 words (kern::deep_max_words)


def full_miner(n_tx: int, pairs_only: bool = False) -> str:
    """Which GPU engine mines every itemset: ``"deep"`` (the headline's persistent wave-per-task
    DFS, kernels/deep.hip, emitting its trie into an HBM arena) whenever the transactions fit its
    tid rows, else ``"levels"`` (the level-wise fused / chunked miner, kernels/levels.hip).
    ``KMLS_FULL_MINER=deep|levels`` overrides (deep still needs n_tx <= 4096)."""
    want = os.environ.get("KMLS_FULL_MINER", "auto").lower()
    if want not in ("auto", "deep", "levels"):
        raise ValueError(f"KMLS_FULL_MINER={want!r}: expected auto, deep or levels")
    fits = 0 < n_tx <= DEEP_MAX_TX and not pairs_only
    if want == "levels" or not fits:
        return "levels"
    return "deep"


def _mine_deep_trie(g, min_support: float, ml: int) -> Dict:
    """Every frequent itemset through the deep miner: emit mode writes each one as a node of an
    HBM arena inside the search, the arena is compacted into a parent-first trie on the device
    (kernels/deep_trie.hip) and copied out in narrow widths (9 B per itemset)."""
    import time
    t0 = time.perf_counter()
    d = g.mine_deep(float(min_support), ml, emit=True)
    t1 = time.perf_counter()
    t = g.deep_arena_trie(1, 0)
    t2 = time.perf_counter()
    if int(t["n"]) != int(d["n_itemsets"]):
        raise RuntimeError(f"deep trie holds {t['n']} nodes for {d['n_itemsets']} itemsets")
    st = {"n_itemsets": int(d["n_itemsets"]), "n_frequent_items": int(d["n_frequent_items"]),
          "max_depth": int(d["max_depth"]), "per_level": list(d["per_level"]),
          "digest": d["digest"], "miner": "deep", "levels_path": "deep-emit",
          "deep_ms": round((t1 - t0) * 1e3, 3), "trie_ms": round((t2 - t1) * 1e3, 3)}
    return {"parent": t["parent"], "item": t["item"], "count": t["count"], "depth": t["depth"],
            "stats": st}


def mine_csr(tx_ptr: np.ndarray, items: np.ndarray, n_items: int, min_support: float,
             max_len: Optional[int] = None, backend: str = "auto", pairs_only: bool = False,
             columns: Optional[Sequence] = None, mfma: bool = False,
             rule_index: bool = False) -> ItemsetTrie:
    """Mine CSR transactions (rows duplicate-free, item ids in [0, n_items)).

    GPU backend: short-transaction data (n_tx <= 4096, the reference's datasets) is mined by the
    deep miner in emit mode (``full_miner``); everything else by the level-wise miner.

    ``rule_index`` (GPU backend): the mining call also builds the rule map on the device
    (``pairs_to_csr``, rows ordered by score desc then consequent name when ``columns`` are
    given); it is returned as ``trie.stats["device_rule_map"]`` (absent if the device could not
    build it, e.g. after a fallback, or on the CPU backends)."""
    if not (0.0 < min_support):
        raise ValueError("`min_support` must be a positive number within the interval `(0, 1]`. "
                         f"Got {min_support}.")
    tx_ptr = np.ascontiguousarray(tx_ptr, dtype=np.int64)
    items = np.ascontiguousarray(items, dtype=np.int32)
    n_tx = len(tx_ptr) - 1
    backend = default_backend() if backend == "auto" else backend
    ml = int(max_len or 0)
    if backend == "oracle":
        X = np.zeros((n_tx, n_items), dtype=bool)
        for t in range(n_tx):
            X[t, items[tx_ptr[t]:tx_ptr[t + 1]]] = True
        recs = _oracle.fpgrowth_oracle(X, min_support, None, max_len)
        if pairs_only:
            recs = [r for r in recs if len(r[1]) <= 2]
        return _trie_from_records(recs, n_tx, min_support, columns)
    if backend == "cpu":
        r = native.load().mine_cpu(tx_ptr, items, int(n_items), float(min_support), ml, 0,
                                   bool(pairs_only))
    elif backend == "gpu":
        g = _gpu_miner()
        g.load_csr(tx_ptr, items, int(n_items))
        if rule_index:
            from ..serve.index import name_tie_rank
            tie = (name_tie_rank([str(c) for c in columns]) if columns is not None else
                   np.arange(int(n_items), dtype=np.int32))
            g.set_tie_rank(np.ascontiguousarray(tie, np.int32))
        # pairs-only == itemsets truncated at 2 items; as max_len it stays on the device-resident
        # path, which is the one that builds the rule map
        if pairs_only:
            ml = 2 if ml == 0 else min(ml, 2)
        if full_miner(n_tx, pairs_only) == "deep" and not mfma:
            idx = None
            if rule_index:  # the deployed rule map = the pair supports: the level-wise call
                # truncated at 2 items builds it on the device (its trie is not downloaded)
                rm = g.mine(float(min_support), 2, False, False, True, False, False, True)
                idx = rm.get("index")
            r = _mine_deep_trie(g, min_support, ml)
            if idx is not None:
                r["index"] = idx
        else:
            r = g.mine(float(min_support), ml, False, True, True, bool(mfma), False,
                       bool(rule_index))
    else:
        raise ValueError(f"unknown backend {backend!r}")
    st = dict(r["stats"])
    st["backend"] = backend
    if rule_index and "index" in r:
        st["device_rule_map"] = r["index"]
    return ItemsetTrie(r["parent"], r["item"], r["count"], r["depth"], n_tx, min_support, st,
                       columns)


def _trie_from_records(recs, n_tx, ms, columns) -> ItemsetTrie:
    # order by size so parents precede children; parent = itemset minus its max item
    sets = sorted(((len(s), tuple(sorted(s)), sup) for sup, s in recs))
    index: Dict[Tuple[int, ...], int] = {}
    par, it, cnt, dep = [], [], [], []
    for k, s, sup in sets:
        p = index[s[:-1]] if k > 1 else -1
        index[s] = len(it)
        par.append(p)
        it.append(s[-1])
        cnt.append(int(round(sup * n_tx)))
        dep.append(k)
    return ItemsetTrie(np.array(par, np.int64), np.array(it, np.int32), np.array(cnt, np.uint32),
                       np.array(dep, np.uint8), n_tx, ms, {"backend": "oracle"}, columns)


def fpgrowth(df, min_support: float = 0.5, use_colnames: bool = False,
             max_len: Optional[int] = None, verbose: int = 0, backend: str = "auto",
             as_trie: bool = False):
    """Drop-in for ``mlxtend.frequent_patterns.fpgrowth`` on a one-hot bool DataFrame/array.

    Returns the mlxtend-shaped DataFrame (or the :class:`ItemsetTrie` if ``as_trie``).
    """
    if hasattr(df, "columns"):
        cols = list(df.columns)
        X = df.values
    else:
        X = np.asarray(df)
        cols = list(range(X.shape[1]))
    if X.dtype != bool:
        if not np.all((X == 0) | (X == 1)):
            raise ValueError("The allowed values for a DataFrame are True, False, 0, 1.")
        X = X.astype(bool)
    T, I = X.shape
    rows, colsx = np.nonzero(X)
    ptr = np.zeros(T + 1, dtype=np.int64)
    np.add.at(ptr, rows + 1, 1)
    ptr = np.cumsum(ptr)
    trie = mine_csr(ptr, colsx.astype(np.int32), I, min_support, max_len, backend,
                    columns=cols if use_colnames else None)
    if as_trie:
        return trie
    return trie.to_dataframe(use_colnames)
