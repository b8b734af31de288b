"""Pure-Python, mlxtend-0.23-faithful reference miner (the parity oracle).

The reference job one-hot encodes playlists with ``mlxtend.preprocessing.TransactionEncoder``
and mines them with ``mlxtend.frequent_patterns.fpgrowth``
(``machine-learning/main.py:262-272``).  mlxtend is not installed in this image (and there is
no network), so this module re-implements the *observable semantics* of those two calls from
SURVEY.md Appendix A, including the two thresholds:

* level 1: an item is frequent iff ``count / T >= min_support`` (float division);
* deeper levels: a conditional item survives iff ``count >= ceil(min_support * T)``.

It also re-implements the reference rule-map builder (``main.py:282-296``) and the serve-time
matcher (``rest_api/app/main.py:224-254``).  Everything here is deliberately slow and simple:
it is the oracle the native CPU miner, the HIP miner and the serving kernels are tested against.
"""
from __future__ import annotations

import itertools
import math
from collections import defaultdict
from typing import Dict, Hashable, Iterable, Iterator, List, Optional, Sequence, Tuple

import numpy as np

__all__ = [
    "transaction_encode",
    "fpgrowth_oracle",
    "frequent_itemsets_bruteforce",
    "rule_map_from_itemsets",
    "rule_map_from_pairs",
    "recommend_oracle",
    "fpgrowth_py_rules_oracle",
    "level2_threshold",
    "level1_is_frequent",
]


# --------------------------------------------------------------------------------------------
# thresholds
# --------------------------------------------------------------------------------------------
def level1_is_frequent(count: int, n_tx: int, min_support: float) -> bool:
    """mlxtend ``setup_fptree``: ``support = count / float(T) >= min_support``."""
    return (count / float(n_tx)) >= min_support


def level2_threshold(n_tx: int, min_support: float) -> int:
    """mlxtend ``fpgrowth``: ``minsup = math.ceil(min_support * T)`` (count threshold)."""
    return int(math.ceil(min_support * n_tx))


def level1_threshold(n_tx: int, min_support: float) -> int:
    """Smallest integer count c with ``c / T >= min_support`` (float semantics of level 1)."""
    c = max(0, int(math.floor(min_support * n_tx)) - 2)
    while not level1_is_frequent(c, n_tx, min_support):
        c += 1
    # step back in case floor() overshot because of rounding
    while c > 0 and level1_is_frequent(c - 1, n_tx, min_support):
        c -= 1
    return c


# --------------------------------------------------------------------------------------------
# TransactionEncoder (mlxtend.preprocessing) semantics
# --------------------------------------------------------------------------------------------
def transaction_encode(transactions: Sequence[Iterable[Hashable]]) -> Tuple[np.ndarray, List]:
    """``TransactionEncoder().fit(tx).transform(tx)``.

    Columns are the sorted set of all items; row r has True at each item of transaction r
    (duplicates collapse).  Returns ``(bool[T, I], columns)``.
    """
    columns = sorted({it for tx in transactions for it in tx})
    col = {c: i for i, c in enumerate(columns)}
    out = np.zeros((len(transactions), len(columns)), dtype=bool)
    for r, tx in enumerate(transactions):
        for it in tx:
            out[r, col[it]] = True
    return out, columns


# --------------------------------------------------------------------------------------------
# FP-tree (pure Python, pointer tree)
# --------------------------------------------------------------------------------------------
class _Node:
    __slots__ = ("item", "count", "parent", "children")

    def __init__(self, item, count=0, parent=None):
        self.item = item
        self.count = count
        self.parent = parent
        self.children: Dict[int, "_Node"] = {}
        if parent is not None:
            parent.children[item] = self

    def path_from_root(self) -> List[int]:
        out = []
        node = self.parent
        while node is not None and node.item is not None:
            out.append(node.item)
            node = node.parent
        out.reverse()
        return out


class _Tree:
    def __init__(self, rank: Dict[int, int]):
        self.root = _Node(None)
        self.header: Dict[int, List[_Node]] = defaultdict(list)  # insertion-ordered
        self.prefix: List[int] = []
        self.rank = rank

    def insert(self, items: Sequence[int], count: int = 1) -> None:
        self.root.count += count
        node = self.root
        i = 0
        for it in items:
            child = node.children.get(it)
            if child is None:
                break
            child.count += count
            node = child
            i += 1
        for it in items[i:]:
            child = _Node(it, count, node)
            self.header[it].append(child)
            node = child

    def single_path(self) -> bool:
        if len(self.root.children) > 1:
            return False
        for nodes in self.header.values():
            if len(nodes) > 1 or len(nodes[0].children) > 1:
                return False
        return True

    def conditional(self, item: int, minsup: int) -> "_Tree":
        paths = []
        cnt: Dict[int, int] = defaultdict(int)
        for node in self.header[item]:
            p = node.path_from_root()
            paths.append((p, node.count))
            for it in p:
                cnt[it] += node.count
        keep = [it for it in cnt if cnt[it] >= minsup]
        keep.sort(key=cnt.get)  # stable sort: ties keep first-seen order
        rank = {it: r for r, it in enumerate(keep)}
        sub = _Tree(rank)
        for p, c in paths:
            sub.insert(sorted([it for it in p if it in rank], key=rank.get, reverse=True), c)
        sub.prefix = self.prefix + [item]
        return sub


def _fpg(tree: _Tree, minsup: int, max_len: Optional[int]) -> Iterator[Tuple[int, List[int]]]:
    items = list(tree.header.keys())
    path = tree.single_path()
    if path:
        top = len(items) + 1 if not max_len else max_len - len(tree.prefix) + 1
        for k in range(1, top):
            for combo in itertools.combinations(items, k):
                yield min(tree.header[i][0].count for i in combo), tree.prefix + list(combo)
    elif not max_len or max_len > len(tree.prefix):
        for it in items:
            yield sum(n.count for n in tree.header[it]), tree.prefix + [it]
    if not path and (not max_len or max_len > len(tree.prefix)):
        for it in items:
            yield from _fpg(tree.conditional(it, minsup), minsup, max_len)


def fpgrowth_oracle(onehot: np.ndarray, min_support: float, columns: Optional[Sequence] = None,
                    max_len: Optional[int] = None) -> List[Tuple[float, frozenset]]:
    """``mlxtend.frequent_patterns.fpgrowth(df, min_support, use_colnames=...)``.

    Returns ``[(support, frozenset(items)), ...]`` in mlxtend's enumeration order (this order
    decides dict insertion order in the reference rule map, hence serve tie order).
    """
    if min_support <= 0.0:
        raise ValueError("`min_support` must be a positive number within the interval `(0, 1]`.")
    X = np.asarray(onehot).astype(bool)
    T = X.shape[0]
    if T == 0:
        return []
    support = X.sum(axis=0) / float(T)
    items = np.nonzero(support >= min_support)[0]
    order = support[items].argsort()  # numpy default quicksort, as mlxtend
    rank = {int(it): r for r, it in enumerate(items[order])}
    tree = _Tree(rank)
    for r in range(T):
        row = [int(i) for i in np.where(X[r])[0] if int(i) in rank]
        row.sort(key=rank.get, reverse=True)
        tree.insert(row)
    minsup = level2_threshold(T, min_support)
    out = []
    for cnt, iset in _fpg(tree, minsup, max_len):
        names = iset if columns is None else [columns[i] for i in iset]
        out.append((cnt / T, frozenset(names)))
    return out


def frequent_itemsets_bruteforce(onehot: np.ndarray, min_support: float,
                                 max_len: Optional[int] = None) -> Dict[frozenset, int]:
    """Level-wise (Apriori) enumeration with the same two thresholds; tiny inputs only.

    Independent of the FP-tree code above, so the two oracles cross-check each other.
    Returns ``{frozenset(column ids): count}``.
    """
    X = np.asarray(onehot).astype(bool)
    T = X.shape[0]
    if T == 0:
        return {}
    cnt1 = X.sum(axis=0)
    f1 = [int(i) for i in range(X.shape[1]) if level1_is_frequent(int(cnt1[i]), T, min_support)]
    res = {frozenset([i]): int(cnt1[i]) for i in f1}
    minsup = level2_threshold(T, min_support)
    level = [(i,) for i in f1]
    k = 1
    while level and (max_len is None or k < max_len):
        nxt = []
        for a_idx in range(len(level)):
            a = level[a_idx]
            for b_idx in range(a_idx + 1, len(level)):
                b = level[b_idx]
                if a[:-1] != b[:-1]:
                    continue
                cand = a + (b[-1],)
                c = int(np.logical_and.reduce(X[:, list(cand)], axis=1).sum())
                if c >= minsup:
                    nxt.append(cand)
                    res[frozenset(cand)] = c
        level = sorted(nxt)
        k += 1
    return res


# --------------------------------------------------------------------------------------------
# reference rule map and matcher
# --------------------------------------------------------------------------------------------
def rule_map_from_itemsets(itemsets: Iterable[Tuple[float, frozenset]]) -> Dict:
    """The reference's ``songs_to_song_sets`` (``machine-learning/main.py:282-296``).

    For every itemset S and song a in S: ``rec[a][b] = max(rec[a][b], support(S))`` for b != a.
    Singletons create keys with empty dicts.  Iteration order follows the input order.
    """
    rec: Dict = {}
    for support, iset in itemsets:
        members = list(iset)
        for a in members:
            row = rec.setdefault(a, {})
            for b in members:
                if b == a:
                    continue
                prev = row.get(b)
                row[b] = support if prev is None else max(prev, support)
    return rec


def rule_map_from_pairs(singles: Iterable[Tuple[Hashable, float]],
                        pairs: Iterable[Tuple[Hashable, Hashable, float]]) -> Dict:
    """Build the same rule map from frequent 1- and 2-itemsets only."""
    rec: Dict = {}
    for a, _ in singles:
        rec.setdefault(a, {})
    for a, b, s in pairs:
        rec.setdefault(a, {})[b] = s
        rec.setdefault(b, {})[a] = s
    return rec


def recommend_oracle(rec: Dict, seeds: Sequence, k: int = 10) -> Optional[List]:
    """``recommend_tracks_for_track`` (``rest_api/app/main.py:224-254``) minus the fallbacks.

    Returns None when no seed is a key (the caller falls back to the static sampler);
    otherwise the top-k names by merged score (stable sort: ties keep insertion order).
    """
    present = [s for s in seeds if s in rec]
    if not present:
        return None
    merged: Dict = defaultdict(int)
    for s in present:
        row = rec[s]
        for r in row:
            merged[r] = max(merged[r], row[r])
    ranked = sorted(merged.items(), key=lambda x: x[1], reverse=True)
    return [name for name, _ in ranked[:k]]


def fpgrowth_py_rules_oracle(transactions: Sequence[Iterable[Hashable]], min_sup_ratio: float,
                             min_conf: float):
    """Semantics of ``fpgrowth_py.fpgrowth(tx, minSupRatio, minConf)`` (dead path J15).

    ``minSup = T * minSupRatio`` (not ceiled); an itemset is frequent iff count >= minSup.
    Rules: every proper non-empty subset A of every frequent itemset S with
    ``conf = count(S) / count(A) > minConf`` → ``[set(A), set(S - A), conf]``.
    Returns None if there is no frequent item (as the library does).
    """
    tx = [set(t) for t in transactions]
    T = len(tx)
    min_sup = T * min_sup_ratio
    onehot, cols = transaction_encode(tx)
    # count threshold "count >= T*ratio" at every level
    X = onehot
    cnt1 = X.sum(axis=0)
    freq: Dict[frozenset, int] = {}
    level = []
    for i in range(X.shape[1]):
        if cnt1[i] >= min_sup:
            freq[frozenset([cols[i]])] = int(cnt1[i])
            level.append((i,))
    while level:
        nxt = []
        for ai in range(len(level)):
            for bi in range(ai + 1, len(level)):
                a, b = level[ai], level[bi]
                if a[:-1] != b[:-1]:
                    continue
                cand = a + (b[-1],)
                c = int(np.logical_and.reduce(X[:, list(cand)], axis=1).sum())
                if c >= min_sup:
                    freq[frozenset(cols[i] for i in cand)] = c
                    nxt.append(cand)
        level = sorted(nxt)
    if not freq:
        return None
    rules = []
    for s, cs in freq.items():
        if len(s) < 2:
            continue
        members = sorted(s, key=repr)
        for r in range(1, len(members)):
            for ante in itertools.combinations(members, r):
                a = frozenset(ante)
                conf = cs / freq[a]
                if conf > min_conf:
                    rules.append([set(a), set(s - a), conf])
    return [set(k) for k in freq], rules
