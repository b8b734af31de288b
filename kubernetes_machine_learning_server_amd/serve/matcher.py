"""Rule matching over a :class:`ModelSnapshot`.

``recommend`` reproduces ``recommend_tracks_for_track`` (``rest_api/app/main.py:224-254``):
present seeds in request order → max-merge → stable sort by score desc → top-K; seeds are not
excluded; all-empty rows → ``[]``; no known seed → static fallback.  The work is done by the
C++ matcher (``_native.RuleIndex.query``) or, batched across requests, by the HIP kernel
``serve_match_topk`` over the HBM-resident index (``serve/batcher.py``).

Static fallback (A8, ``main.py:205-222``): a seeded sample of K best tracks.  The reference
seeds the GLOBAL RNG with the process-salted ``hash(tuple(sorted(seeds)))`` (different on each
replica, Appendix B.8) and raises if fewer than K best tracks exist (B.5).  Here the seed is a
stable FNV-1a 64 hash of the sorted seeds, a private ``random.Random`` is used, and K is clamped.
The native serving front (csrc/host/http_front.cpp) computes the same seed and reproduces
``random.Random(seed).sample`` bit-exactly, so both paths return the same fallback list.
"""
from __future__ import annotations

import random
from typing import List, Optional, Sequence

import numpy as np

from .state import ModelSnapshot

NO_RECOMMENDATIONS = "No recommendations available at the moment"


_FNV_OFFSET, _FNV_PRIME, _M64 = 0xCBF29CE484222325, 0x100000001B3, (1 << 64) - 1


def stable_seed(seeds: Sequence[str]) -> int:
    """FNV-1a 64 of ``"\\x1f".join(sorted(seeds))`` in UTF-8 (== _native.fallback_seed)."""
    h = _FNV_OFFSET
    for b in "\x1f".join(sorted(seeds)).encode("utf-8"):
        h = ((h ^ b) * _FNV_PRIME) & _M64
    return h


def static_recommendation(snap: Optional[ModelSnapshot], seeds: Sequence[str], k: int) -> List[str]:
    if snap is None or not snap.best_tracks:
        return [NO_RECOMMENDATIONS]
    rng = random.Random(stable_seed(seeds))
    names = snap.best_track_names
    return rng.sample(names, k=min(k, len(names)))


def seed_ids(snap: ModelSnapshot, seeds: Sequence[str]) -> np.ndarray:
    n2i = snap.index.name_to_id
    return np.fromiter((n2i.get(s, -1) for s in seeds), dtype=np.int32, count=len(seeds))


def recommend_cpu(snap: ModelSnapshot, seeds: Sequence[str], k: int) -> Optional[List[str]]:
    """None = no seed is a key (caller falls back); else the ordered top-k names."""
    ids = snap.index.native().query(seed_ids(snap, seeds), k)
    if ids is None:
        return None
    names = snap.index.names
    return [names[i] for i in ids]


def decode_batch(snap: ModelSnapshot, ids: np.ndarray, n: np.ndarray, row: int) -> Optional[List[str]]:
    m = int(n[row])
    if m < 0:
        return None
    names = snap.index.names
    return [names[i] for i in ids[row, :m]]
