"""Count-only full FP-Growth mining of ONE dataset split over the GPUs of a node.

The reference mines every frequent itemset of every size (``machine-learning/main.py:272``) and
sweeps min_support downwards (``main.py:450-473``).  At the BASELINE config-2 family (ds1 at
0.01-0.02) the output is 1e9-1e10 itemsets: every itemset and its support is computed, the
per-size counts and the content digest (``kmls/digest.hpp``, equal to the digest of the full
trie) are kept, nothing is materialised (``GpuMiner.mine_deep``, ``csrc/kernels/deep.hip``).

Split over ranks (strong scaling): every rank builds the same level-2 classes on its own GPU
(deterministic), the level-3 tasks are ordered by an estimated cost and dealt to the ranks in a
snake order (``csrc/host/deep_run.hip``), and the per-size counts and digest sums are all-reduced
(the digest xors all-gathered), so every rank ends with the result of the whole problem.  The
combine runs through one of:

* ``"rccl"``  — the native communicator (``csrc/host/comm_rccl.cpp``: RCCL over xGMI, issued on
  the miner's stream inside ``mine_deep``);
* ``"host"``  — the native host shared-memory communicator (ranks sharing one GPU, CPU tests);
* ``"torch"`` — ``torch.distributed`` on the job's process group (RCCL on an ``nccl`` group,
  gloo otherwise): one 66-word all-reduce + one all-gather per call, after ``mine_deep``
  returned the rank's partial.
"""
from __future__ import annotations

import os
import math
import random
import time
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from ..ops import native

try:
    import torch
    import torch.distributed as dist
except Exception:  # pragma: no cover
    torch = None
    dist = None

_U64 = 1 << 64


def _s64(v: int) -> int:
    v %= _U64
    return v - _U64 if v >= (1 << 63) else v


def _all_gather_int(v: int, world: int, device: int = 0) -> List[int]:
    dev = (torch.device("cuda", device) if dist.get_backend() == "nccl"
           else torch.device("cpu"))
    x = torch.tensor([v], dtype=torch.int64, device=dev)
    xs = torch.empty(world, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(xs, x)
    return [int(a) for a in xs.cpu().tolist()]


def combine_partials(parts: List[Dict]) -> Dict:
    """Whole-problem result from per-rank partials (what the collectives compute)."""
    per = [0] * 64
    dsum = dxor = cands = 0
    for p in parts:
        for d, v in enumerate(p["per_level"]):
            per[d] += int(v)
        dsum = (dsum + int(p["digest"][:16], 16)) % _U64
        dxor ^= int(p["digest"][16:], 16)
        cands += int(p["candidates"])
    return _finish(dict(parts[0]), per, dsum, dxor, cands)


def _finish(d: Dict, per: List[int], dsum: int, dxor: int, cands: int) -> Dict:
    while len(per) > 2 and per[-1] == 0:
        per.pop()
    d["per_level"] = per
    d["n_itemsets"] = sum(per[1:])
    d["max_depth"] = max([i for i, v in enumerate(per) if v and i > 0], default=0)
    d["digest"] = f"{dsum % _U64:016x}{dxor % _U64:016x}"
    d["candidates"] = cands
    return d


def allreduce_partial(d: Dict, world: int, device: int = 0) -> Dict:
    """Whole-problem result from this rank's partial through torch.distributed: one 66-word
    int64 all-reduce (per-size counts, digest sum, candidates; wrapping sums are the mod-2^64
    sums) and one all-gather of the digest xor.  RCCL on an nccl group, gloo otherwise."""
    dev = (torch.device("cuda", device) if dist.get_backend() == "nccl"
           else torch.device("cpu"))
    per = list(d["per_level"]) + [0] * (64 - len(d["per_level"]))
    red = torch.tensor([_s64(v) for v in per] + [_s64(int(d["digest"][:16], 16)),
                                                 int(d.get("candidates", 0))],
                       dtype=torch.int64, device=dev)
    dist.all_reduce(red)
    x = torch.tensor([_s64(int(d["digest"][16:], 16))], dtype=torch.int64, device=dev)
    xs = [torch.empty_like(x) for _ in range(world)]
    dist.all_gather(xs, x)
    v = [int(t) % _U64 for t in red.cpu().tolist()]
    dxor = 0
    for t in xs:
        dxor ^= int(t.item()) % _U64
    return _finish(dict(d), v[:64], v[64], dxor, v[65])


class DeepMiner:
    def __init__(self, tx_ptr, items, n_items: int, device: int = 0, rank: int = 0,
                 world: int = 1, comm_backend: Optional[str] = None, **opts):
        self.N = native.require_gpu()
        self.rank, self.world, self.device = rank, world, device
        self.opts = dict(opts)
        self.comm = None
        self.comm_backend = None
        if world > 1:
            backend = comm_backend or os.environ.get("KMLS_COMM") or (
                "rccl" if dist is not None and dist.is_initialized() and
                dist.get_backend() == "nccl" else "host")
            if backend not in ("rccl", "host", "torch"):
                raise ValueError(f"DeepMiner: unknown comm backend {backend!r}")
            if backend != "torch":
                make_uid = (self.N.host_comm_unique_id if backend == "host"
                            else self.N.comm_unique_id)
                uid = [make_uid() if rank == 0 else b"\0" * 128]
                dist.broadcast_object_list(uid, src=0)
                self.comm = self.N.Comm(rank, world, uid[0], device, backend)
            self.comm_backend = backend
        self.g = self.N.GpuMiner(device)
        self.g.load_csr(tx_ptr, items, n_items)

    def mine(self, min_support: float, max_len: int = 0) -> Dict:
        """Whole-problem result on every rank (per_level, n_itemsets, digest, ...)."""
        d = self.g.mine_deep(min_support, max_len, self.rank, self.world, self.comm,
                             **self.opts)
        if self.comm_backend == "torch":
            d = self._combine_torch(d)
        return d

    def mine_trie(self, min_support: float, max_len: int = 0) -> Tuple[Dict, Optional[Dict]]:
        """Every frequent itemset as a trie, mined by the split (emit mode) and gathered on rank
        0: ``(whole-problem result, trie arrays on rank 0 / None elsewhere)``.

        Each rank's arena is compacted on its GPU (``deep_arena_trie``): rank 0 exports every
        size (levels 1-2 are the dense ids [0, P12), P12 = F + frequent pairs, the same arena ids
        on every rank), a rank r > 0 exports its share (sizes >= 3) with its own node ids shifted
        past P12 and its size-2 parents kept as arena ids.  Rank 0 concatenates the shares in
        rank order and moves each share's ids to its offset; parents stay before children (a
        share's parents are in the share or in rank 0's levels 1-2)."""
        d = self.g.mine_deep(min_support, max_len, self.rank, self.world, self.comm, emit=True,
                             **self.opts)
        if self.comm_backend == "torch":
            d = self._combine_torch(d)
        per = list(d["per_level"]) + [0, 0, 0]
        p12 = int(per[1]) + int(per[2])
        t = self.g.deep_arena_trie(1 if self.rank == 0 else 3, 0 if self.rank == 0 else p12)
        fields = ("parent", "item", "count", "depth")
        if self.world == 1:
            return d, {k: t[k] for k in fields}
        from .dist_miner import gather_arrays
        dtypes = {k: np.asarray(t[k]).dtype for k in fields}
        # uint8 views: every collective backend carries bytes (RCCL has no 16-bit integers)
        # (one field per call: gather_arrays sizes every field by the first one's length)
        raw = {k: gather_arrays({k: np.ascontiguousarray(t[k]).view(np.uint8)}, self.rank,
                                self.world) for k in fields}
        raw = {k: (v[k] if v is not None else None) for k, v in raw.items()}
        sizes = [int(x) for x in _all_gather_int(int(t["n"]), self.world, self.device)]
        if self.rank != 0:
            return d, None
        out = {k: raw[k].view(dtypes[k]).copy() for k in fields}
        par = out["parent"]
        if sum(sizes) >= (1 << 31):
            raise RuntimeError("deep trie: 2^31 nodes (i32 parents)")
        off = sizes[0]
        for r in range(1, self.world):
            blk = par[off:off + sizes[r]]
            blk[blk >= p12] += off - p12
            off += sizes[r]
        if off != int(d["n_itemsets"]):
            raise RuntimeError(f"deep trie: gathered {off} nodes for {d['n_itemsets']} itemsets")
        return d, out

    def _combine_torch(self, d: Dict) -> Dict:
        return allreduce_partial(d, self.world, self.device)

    def synchronize(self) -> None:
        self.g.synchronize()


def estimate_total(g, min_support: float, world: int, samples: int, seed: int = 0,
                   max_len: int = 0, budget_s: float = 0.0, ranks: Optional[Sequence[int]] = None,
                   **opts) -> Dict:
    """Estimate of a full mining result too large to count whole on one GPU in a bench step
    (BASELINE config 2, ds1 @ 0.01: > 4.7e11 itemsets up to size 9 alone).

    The level-3 tasks are dealt to `world` virtual ranks exactly as a real split deals them
    (cost-ordered snake deal, so every rank's share is a stratified slice of the task costs);
    `samples` ranks drawn uniformly without replacement are mined EXACTLY (``mine_deep`` with
    that rank/world, no communicator), and the total is ``world x mean`` of their counts: an
    unbiased estimator, with the standard error from the sample variance and the
    finite-population correction.  Per-size counts are estimated the same way.  Sampling stops
    early once `budget_s` seconds have been spent (at least two samples).  Reference: the
    reference mines every size (``machine-learning/main.py:272``)."""
    rng = random.Random(seed)
    pick = list(ranks) if ranks is not None else rng.sample(range(world), min(samples, world))
    xs, per, secs, done = [], [], [], []
    t_all = time.perf_counter()
    for r in pick:
        t = time.perf_counter()
        d = g.mine_deep(min_support, max_len, int(r), int(world), None, **opts)
        secs.append(time.perf_counter() - t)
        xs.append(int(d["n_itemsets"]))
        per.append([int(v) for v in d["per_level"]])
        done.append(int(r))
        if budget_s and len(xs) >= 2 and time.perf_counter() - t_all > budget_s:
            break
    k = len(xs)
    fpc = 1.0 - k / world

    def est(vals):
        m = sum(vals) / k
        var = sum((v - m) ** 2 for v in vals) / (k - 1) if k > 1 else float("nan")
        return world * m, world * math.sqrt(max(var, 0.0) * fpc / k) if k > 1 else float("nan")

    n_est, n_se = est(xs)
    depth = max(len(p) for p in per)
    per_est = []
    for dd in range(1, depth):
        e, s = est([p[dd] if dd < len(p) else 0 for p in per])
        per_est.append({"size": dd, "estimate": round(e), "se": round(s)})
    t_est, t_se = est(secs)
    return {"method": "snake-dealt virtual ranks, simple random sample, world x mean",
            "world": world, "samples": k, "ranks": done, "min_support": min_support,
            "max_len": max_len, "n_itemsets_estimate": round(n_est),
            "n_itemsets_se": round(n_se), "rel_se": round(n_se / n_est, 4) if n_est else None,
            "per_size": per_est, "one_gpu_s_estimate": round(t_est, 1),
            "one_gpu_s_se": round(t_se, 1), "sample_s": [round(x, 3) for x in secs],
            "sample_n": xs}
