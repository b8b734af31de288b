"""Multi-GPU FP-Growth: one process per GPU, torch.distributed over RCCL (xGMI).

The reference job is single-process (``machine-learning/main.py:421-484``; SURVEY §2.E lists
no parallelism).  Here the mining step is split across the N GPUs of a node:

1. **transaction-DP supports** — rank r owns transactions ``[r*Ts, (r+1)*Ts)`` (Ts a multiple
   of 256 so shard boundaries fall on 4-word bitmap boundaries).  Per-item supports are counted
   on each shard by the HIP histogram kernel and combined with one RCCL ``all_reduce`` (the
   support vector is small — latency-bound, one collective).
2. **bitmap re-shard (all-gather)** — every rank encodes the tid-bitmaps of the frequent items
   for its own transactions ([F][Ws] words) and one ``all_gather_into_tensor`` assembles the
   replicated [F][N*Ws] bitmap (an int64 transpose on the device afterwards).  One large
   collective instead of many small ones: xGMI rings are per-link bound, so fewer, bigger
   messages.
3. **item-sharded DFS** — the equivalence-class tree is split at the root: rank r expands the
   top-level classes it owns (PFP-style group-dependent sharding).  Ownership is a
   deterministic LPT partition of the root classes by estimated cost (computed identically on
   every rank from the level-2 co-occurrence counts, so no extra collective is needed).
4. **result** — each rank keeps its sub-trie; the global itemset count is one ``all_reduce``;
   ``gather_trie`` concatenates sub-tries on rank 0 when the caller needs them (the job).

With N == 1 every collective is skipped and the native single-GPU ``mine`` path runs.
"""
from __future__ import annotations

import os
import time
from typing import Dict, List, Optional, Tuple

import numpy as np

from ..ops import native

try:  # torch is only needed for the multi-GPU path
    import torch
    import torch.distributed as dist
except Exception:  # pragma: no cover
    torch = None
    dist = None


def shard_bounds(n_tx: int, world: int, rank: int, align: int = 256) -> Tuple[int, int, int]:
    """(lo, hi, Ts): rank's transaction range; Ts is the aligned per-rank stride."""
    ts = -(-n_tx // world)
    ts = -(-ts // align) * align
    lo = min(n_tx, rank * ts)
    hi = min(n_tx, lo + ts)
    return lo, hi, ts


def lpt_partition(cost: np.ndarray, world: int) -> np.ndarray:
    """Longest-processing-time-first assignment of root classes to ranks (deterministic)."""
    owner = np.zeros(len(cost), dtype=np.int32)
    if world <= 1:
        return owner
    order = np.argsort(-cost, kind="stable")
    load = np.zeros(world, dtype=np.float64)
    for a in order:
        r = int(np.argmin(load))
        owner[a] = r
        load[r] += float(cost[a])
    return owner


def root_costs(gram: np.ndarray, minsup: int) -> np.ndarray:
    """Estimated subtree cost of each root class from level-2 counts: n_a^2 + 1 where n_a is the
    number of frequent extensions of item a (its level-3 candidate count ~ n_a^2 / 2)."""
    F = gram.shape[0]
    upper = np.triu(gram >= minsup, k=1)
    n = upper.sum(axis=1).astype(np.float64)
    return n * n + 1.0


class DistMiner:
    """Mine one resident dataset repeatedly (the bench step / the job's mining call)."""

    def __init__(self, tx_ptr: np.ndarray, items: np.ndarray, n_items: int, min_support: float,
                 device: int = 0, max_len: int = 0, mfma: bool = False,
                 arena_bytes: int = 0):
        self.world = dist.get_world_size() if (dist is not None and dist.is_initialized()) else 1
        self.rank = dist.get_rank() if self.world > 1 else 0
        self.n_tx = len(tx_ptr) - 1
        self.n_items = int(n_items)
        self.min_support = float(min_support)
        self.max_len = int(max_len)
        self.mfma = bool(mfma)
        self.device = device
        N = native.require_gpu()
        if self.world > 1:
            torch.cuda.set_device(device)
            self.stream = torch.cuda.Stream(device=device)
            self.g = N.GpuMiner(device, arena_bytes, self.stream.cuda_stream)
        else:
            self.stream = None
            self.g = N.GpuMiner(device, arena_bytes, 0)
        lo, hi, ts = shard_bounds(self.n_tx, self.world, self.rank)
        self.lo, self.hi, self.ts = lo, hi, ts
        sp = tx_ptr[lo:hi + 1]
        self.g.load_csr(np.ascontiguousarray(sp - sp[0], dtype=np.int64),
                        np.ascontiguousarray(items[sp[0]:sp[-1]], dtype=np.int32), self.n_items)
        self.last: Dict = {}

    # ------------------------------------------------------------------------------------
    def step(self, download: bool = True) -> Dict:
        if self.world == 1:
            r = self.g.mine(self.min_support, self.max_len, False, download, True, self.mfma)
            st = dict(r["stats"])
            st["global_itemsets"] = int(st["n_itemsets"])
            self.last = r
            return {"stats": st, "trie": r}
        return self._step_dist(download)

    def _step_dist(self, download: bool) -> Dict:
        g = self.g
        dev = torch.device("cuda", self.device)
        t0 = time.perf_counter()
        ph: Dict[str, float] = {}
        with torch.cuda.stream(self.stream):
            counts = torch.empty(self.n_items, dtype=torch.int32, device=dev)
            g.item_support(counts.data_ptr())
            dist.all_reduce(counts, op=dist.ReduceOp.SUM)  # RCCL over xGMI
            host_counts = counts.cpu().numpy().view(np.uint32)
            F = g.select(host_counts, self.n_tx, self.min_support)
            ph["supports_allreduce"] = time.perf_counter() - t0
            ws = self.ts // 64
            wp = ws * self.world
            if F == 0:
                return {"stats": {"n_itemsets": 0, "global_itemsets": 0, "n_frequent_items": 0}}
            local = torch.zeros((F, ws), dtype=torch.int64, device=dev)
            g.encode_bitmaps(local.data_ptr(), ws, 0)
            gathered = torch.empty((self.world, F, ws), dtype=torch.int64, device=dev)
            dist.all_gather_into_tensor(gathered, local)
            bm = gathered.permute(1, 0, 2).reshape(F, wp).contiguous()
            del gathered, local
            ph["bitmap_allgather"] = time.perf_counter() - t0
            # ownership from level-2 counts (identical on every rank)
            gram = torch.empty((F, F), dtype=torch.int32, device=dev)
            g.pair_counts(bm.data_ptr(), wp, gram.data_ptr(), self.mfma)
            _, _, minsup = g.frequent()
            gh = gram.cpu().numpy().view(np.uint32)
            owner = lpt_partition(root_costs(gh, int(minsup)), self.world)
            owned = (owner == self.rank).astype(np.uint8)
            del gram
            ph["partition"] = time.perf_counter() - t0
            self.stream.synchronize()
            r = g.mine_bitmaps(bm.data_ptr(), wp, self.min_support, self.max_len, False, owned,
                               self.rank == 0, download, True, self.mfma)
            ph["mine"] = time.perf_counter() - t0
            tot = torch.tensor([int(r["stats"]["n_itemsets"])], dtype=torch.int64, device=dev)
            dist.all_reduce(tot, op=dist.ReduceOp.SUM)
            st = dict(r["stats"])
            st["global_itemsets"] = int(tot.item())
            st["host_phases_s"] = ph
        self.last = r
        return {"stats": st, "trie": r}


def gather_trie(r: Dict, rank: int, world: int, n_frequent: int) -> Optional[Dict[str, np.ndarray]]:
    """Concatenate per-rank sub-tries on rank 0 (level-1 nodes 0..F-1 are shared; every rank's
    local ids >= F are rebased)."""
    if world == 1:
        return {k: r[k] for k in ("parent", "item", "count", "depth")}
    parts = [None] * world
    mine = {k: np.asarray(r[k]) for k in ("parent", "item", "count", "depth")}
    dist.all_gather_object(parts, mine)
    if rank != 0:
        return None
    F = n_frequent
    out = {k: [parts[0][k][:F]] for k in mine}
    base = F
    for p in parts:
        n = len(p["item"]) - F
        if n <= 0:
            continue
        par = p["parent"][F:].copy()
        loc = par >= F
        par[loc] += base - F
        out["parent"].append(par)
        for k in ("item", "count", "depth"):
            out[k].append(p[k][F:])
        base += n
    return {k: np.concatenate(v) for k, v in out.items()}
