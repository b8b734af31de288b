"""Integer rule index: the reference's ``recommendations.pickle`` as CSR arrays.

Reference format (``machine-learning/main.py:282-296,479``):
``dict[track_name, dict[track_name, float support]]`` — keys are all frequent songs (some with
``{}``), ``rec[a][b] = support({a, b})`` (the max over itemsets containing both equals the pair
support by anti-monotonicity).

Here the same information is a CSR over integer item ids: ``row_ptr/cons/score`` plus an
``is_key`` mask (a key with an empty row is different from "unknown song":
``rest_api/app/main.py:235-238``).  Row order is the dict's inner insertion order, which decides
serve-time tie order; indices built from a mined trie use (score desc, consequent name asc).
The same arrays feed the C++ matcher (``_native.RuleIndex``) and the HBM-resident HIP index
(``_native.GpuRuleIndex``) and serialise to ``rules.idx`` (npz) next to the pickle.
"""
from __future__ import annotations

import dataclasses
import io
import pathlib
from typing import Dict, Hashable, List, Optional, Sequence

import numpy as np

from ..ops import native
from ..utils.atomic_io import atomic_write_bytes


@dataclasses.dataclass
class RuleIndexData:
    n_items: int
    row_ptr: np.ndarray   # int64[n_items + 1]
    cons: np.ndarray      # int32[nnz]
    score: np.ndarray     # float64[nnz]
    is_key: np.ndarray    # uint8[n_items]
    names: Optional[List[str]] = None

    def __post_init__(self):
        self._name_to_id: Optional[Dict[str, int]] = None
        self._native = None

    # ---------------------------------------------------------------------------------
    @property
    def name_to_id(self) -> Dict[str, int]:
        if self._name_to_id is None:
            self._name_to_id = {n: i for i, n in enumerate(self.names or [])}
        return self._name_to_id

    @property
    def n_keys(self) -> int:
        return int(self.is_key.sum())

    @property
    def nnz(self) -> int:
        return int(len(self.cons))

    def native(self):
        if self._native is None:
            self._native = native.load().RuleIndex(
                int(self.n_items), np.ascontiguousarray(self.row_ptr, np.int64),
                np.ascontiguousarray(self.cons, np.int32), np.ascontiguousarray(self.score, np.float64),
                np.ascontiguousarray(self.is_key, np.uint8))
        return self._native

    def row(self, i: int):
        s, e = int(self.row_ptr[i]), int(self.row_ptr[i + 1])
        return self.cons[s:e], self.score[s:e]

    def to_rec_dict(self) -> Dict[str, Dict[str, float]]:
        """The reference pickle object (insertion order = key id order, row order)."""
        names = self.names or [str(i) for i in range(self.n_items)]
        rec: Dict[str, Dict[str, float]] = {}
        rp, cons, sc = self.row_ptr, self.cons, self.score
        for i in np.nonzero(self.is_key)[0]:
            s, e = int(rp[i]), int(rp[i + 1])
            rec[names[i]] = {names[int(c)]: float(v) for c, v in zip(cons[s:e], sc[s:e])}
        return rec

    @classmethod
    def from_rec_dict(cls, rec: Dict[Hashable, Dict[Hashable, float]],
                      extra_names: Sequence[str] = ()) -> "RuleIndexData":
        """Index an arbitrary reference-format dict, preserving its inner order exactly."""
        names: List = list(rec.keys())
        nid = {n: i for i, n in enumerate(names)}
        for row in rec.values():
            for c in row:
                if c not in nid:
                    nid[c] = len(names)
                    names.append(c)
        for n in extra_names:
            if n not in nid:
                nid[n] = len(names)
                names.append(n)
        n_items = len(names)
        row_ptr = np.zeros(n_items + 1, np.int64)
        cons: List[int] = []
        score: List[float] = []
        is_key = np.zeros(n_items, np.uint8)
        for k, row in rec.items():
            i = nid[k]
            is_key[i] = 1
        # rows in id order
        for i in range(n_items):
            nm = names[i]
            if is_key[i]:
                row = rec[nm]
                for c, v in row.items():
                    cons.append(nid[c])
                    score.append(float(v))
            row_ptr[i + 1] = len(cons)
        return cls(n_items, row_ptr, np.asarray(cons, np.int32), np.asarray(score, np.float64),
                   is_key, [str(n) for n in names])

    # ---------------------------------------------------------------------------------
    def save(self, path) -> None:
        """Binary index (``rules.idx``): CSR arrays + string table, loadable without pickle."""
        buf = io.BytesIO()
        names = np.asarray(self.names if self.names is not None else [], dtype=object)
        enc = np.frombuffer("\x00".join(map(str, names)).encode("utf-8"), dtype=np.uint8)
        np.savez(buf, n_items=np.int64(self.n_items), row_ptr=self.row_ptr, cons=self.cons,
                 score=self.score, is_key=self.is_key, names_utf8=enc,
                 n_names=np.int64(len(names)))
        # tmp + fsync + rename, like the pickles: a reader never sees a truncated index
        atomic_write_bytes(path, buf.getvalue())

    @classmethod
    def load(cls, path) -> "RuleIndexData":
        z = np.load(pathlib.Path(path), allow_pickle=False)
        n_names = int(z["n_names"])
        names = bytes(z["names_utf8"]).decode("utf-8").split("\x00") if n_names else None
        return cls(int(z["n_items"]), z["row_ptr"], z["cons"], z["score"], z["is_key"], names)


def name_tie_rank(names: Sequence[str]) -> np.ndarray:
    """Rank of every item's name in sorted order (stable: equal names keep id order) — the
    tie key of index rows, here and in the device rule-map kernel (``GpuMiner.set_tie_rank``)."""
    n = len(names)
    r = np.empty(n, np.int32)
    r[np.argsort(np.asarray(names, dtype=object), kind="stable")] = np.arange(n, dtype=np.int32)
    return r


def index_from_device_csr(ix: Dict, n_items: int, single_ids: np.ndarray, n_tx: int,
                          names: Optional[Sequence[str]] = None) -> RuleIndexData:
    """RuleIndexData from the device-built rule map (``mine(..., rule_index=True)["index"]``):
    rows are already in index order; keys are the frequent single items."""
    is_key = np.zeros(n_items, np.uint8)
    is_key[np.asarray(single_ids, np.int64)] = 1
    score = np.asarray(ix["count"], np.float64) / float(n_tx)
    return RuleIndexData(int(n_items), np.array(ix["row_ptr"], np.int64),
                         np.array(ix["cons"], np.int32), score, is_key,
                         list(names) if names is not None else None)


def build_index_from_pairs(n_items: int, single_ids: np.ndarray, pair_a: np.ndarray,
                           pair_b: np.ndarray, pair_count: np.ndarray, n_tx: int,
                           names: Optional[Sequence[str]] = None) -> RuleIndexData:
    """Keys = frequent single items; rows = frequent pairs in both directions; score =
    count / T (float64, as the reference's ``row.support``).  Row order: score desc, then
    consequent name (or id) asc — a deterministic stand-in for mlxtend's enumeration order."""
    a = np.asarray(pair_a, np.int64)
    b = np.asarray(pair_b, np.int64)
    c = np.asarray(pair_count, np.int64)
    src = np.concatenate([a, b])
    dst = np.concatenate([b, a])
    cnt = np.concatenate([c, c])
    if names is not None:
        name_rank = name_tie_rank(names).astype(np.int64)
        tie = name_rank[dst] if len(dst) else dst
    else:
        tie = dst
    order = np.lexsort((tie, -cnt, src))
    src, dst, cnt = src[order], dst[order], cnt[order]
    row_ptr = np.zeros(n_items + 1, np.int64)
    np.cumsum(np.bincount(src, minlength=n_items), out=row_ptr[1:])
    is_key = np.zeros(n_items, np.uint8)
    is_key[np.asarray(single_ids, np.int64)] = 1
    score = cnt.astype(np.float64) / float(n_tx)
    return RuleIndexData(int(n_items), row_ptr, dst.astype(np.int32), score, is_key,
                         list(names) if names is not None else None)


def build_index_from_trie(parent, item, count, depth, n_tx: int, n_items: int,
                          names: Optional[Sequence[str]] = None) -> RuleIndexData:
    parent = np.asarray(parent)
    item = np.asarray(item)
    depth = np.asarray(depth)
    count = np.asarray(count)
    m1 = depth == 1
    m2 = depth == 2
    return build_index_from_pairs(n_items, item[m1], item[parent[m2]], item[m2], count[m2],
                                  n_tx, names)
