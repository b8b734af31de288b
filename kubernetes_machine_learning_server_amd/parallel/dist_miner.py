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

**Replicated mode** (``mode="replicate"``, the default for small data on N > 1 GPUs, e.g. the
ds1/ds2 headline): the whole CSR is tiny (240k rows), so every rank holds all of it and runs the
device-resident single-GPU prologue (supports, selection, bitmaps, level-2 gram — no
collective), then expands only the root classes that a device-side snake partition of the
estimated class costs assigns to it (``GpuMiner.mine_partition``).  One collective per step
(the itemset-count all-reduce) instead of four plus host round trips.

**Transaction-DP mode** (``mode="tx"``, the default for T >= 4M — BASELINE configs 3 and 5;
``backend="cpu"`` runs the same level loop natively on the host over the shared-memory
communicator, the multi-process CPU test tier):
replicating [F][T/64] bitmaps stops paying when T is large (100M transactions x 756 frequent
items = 9.4 GB per GPU), so each rank keeps only its own shard's bitmap words and the C++
level loop all-reduces every level's candidate counts through a native RCCL communicator
(``csrc/host/comm_rccl.cpp``) on the miner's stream — no Python round trip per level.  The
per-item supports are counted in tiles whose all-reduces run on a side stream while the next
tile's histogram runs (the overlap the north star asks for).  Every rank ends with the same
global trie; rank 0 downloads it.

**Dataset-parallel mode** (``mode="local"``): each rank mines its own whole dataset with the
native single-GPU path and no collective — the job's min_support sweep split over the GPUs
(``job.main.run_support_sweep``) and the weak-scaled bench (one dataset per GPU).  A ds-sized problem is a
0.3 ms chain of dependent level launches, so N independent datasets is the form of it that
scales with GPUs; ``replicate`` stays the strong-scaled form of one dataset.
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


def comm_backend() -> str:
    """Native communicator of the tx-DP level loop: ``KMLS_COMM`` (``rccl`` | ``host``); default
    RCCL when the process group runs on it, else the host shared-memory backend (gloo process
    groups, several ranks sharing one GPU)."""
    env = os.environ.get("KMLS_COMM", "").strip().lower()
    if env in ("rccl", "host"):
        return env
    if dist is not None and dist.is_initialized() and dist.get_backend() == "nccl":
        return "rccl"
    return "host"


def shard_bounds(n_tx: int, world: int, rank: int, align: int = 256) -> Tuple[int, int, int]:
    """(lo, hi, Ts): rank's transaction range; Ts is the aligned per-rank stride."""
    ts = -(-n_tx // world)
    ts = -(-ts // align) * align
    lo = min(n_tx, rank * ts)
    hi = min(n_tx, lo + ts)
    return lo, hi, ts


def lpt_partition(cost: np.ndarray, world: int) -> np.ndarray:
    """Balanced, deterministic assignment of root classes to ranks.

    Classes are sorted by estimated cost (desc) and dealt in snake order (0..N-1, N-1..0, ...):
    an O(F log F) vectorised stand-in for LPT that keeps the per-step host cost in the tens of
    microseconds (an interpreted LPT loop costs ~1 ms at F≈800).  Identical on every rank.
    """
    F = len(cost)
    owner = np.zeros(F, dtype=np.int32)
    if world <= 1 or F == 0:
        return owner
    order = np.argsort(-np.asarray(cost, dtype=np.float64), kind="stable")
    k = np.arange(F)
    rnd, pos = k // world, k % world
    owner[order] = np.where(rnd % 2 == 0, pos, world - 1 - pos).astype(np.int32)
    return owner


def root_costs(gram, minsup: int) -> np.ndarray:
    """Estimated subtree cost of each root class from level-2 counts: n_a^2 + 1, n_a = number
    of frequent extensions of item a (its level-3 candidates ~ n_a^2 / 2).  Accepts a torch
    tensor (reduced on its device; only F values cross to the host) or a numpy array."""
    if torch is not None and isinstance(gram, torch.Tensor):
        F = gram.shape[0]
        m = (gram.to(torch.int64) & 0xFFFFFFFF) >= minsup
        n = torch.triu(m, diagonal=1).sum(dim=1).to(torch.float64)
        return (n * n + 1.0).cpu().numpy()
    upper = np.triu(np.asarray(gram) >= minsup, k=1)
    n = upper.sum(axis=1).astype(np.float64)
    return n * n + 1.0


class _GpuOps:
    """Device ops of the protocol on one MI355X (HIP kernels; tensors in HBM; RCCL)."""

    def __init__(self, dm: "DistMiner", tx_ptr, items, arena_bytes: int):
        N = native.require_gpu()
        self.dev = torch.device("cuda", dm.device)
        self.comm = None
        if dm.mode == "replicate":
            torch.cuda.set_device(dm.device)
            self.stream = None
            self.g = N.GpuMiner(dm.device, arena_bytes, 0)
        elif dm.mode == "tx":
            torch.cuda.set_device(dm.device)
            backend = comm_backend()
            make_uid = N.host_comm_unique_id if backend == "host" else N.comm_unique_id
            # KMLS_COMM_FORCE=1: a real one-rank RCCL communicator (the RCCL path's test hook)
            forced = dm.world == 1 and backend == "rccl" and os.environ.get("KMLS_COMM_FORCE") == "1"
            uid = [make_uid() if dm.rank == 0 and (dm.world > 1 or forced) else b"\0" * 128]
            if dm.world > 1:
                dist.broadcast_object_list(uid, src=0)
            self.comm = N.Comm(dm.rank, dm.world, uid[0], dm.device, backend)
            self.stream = None
            self.g = N.GpuMiner(dm.device, arena_bytes, 0)
        elif (dm.world > 1 and dm.mode != "local") or dm.force_protocol \
                or dm.mode in ("item", "shard"):
            # every torch op of the protocol (allocations, fills, collectives) and every native
            # kernel run on ONE stream, so they are ordered without extra synchronisation
            torch.cuda.set_device(dm.device)
            self.stream = torch.cuda.Stream(device=dm.device)
            self.g = N.GpuMiner(dm.device, arena_bytes, self.stream.cuda_stream)
            if dm.mode == "shard" and os.environ.get("KMLS_SHARD_NATIVE", "1") != "0":
                # the native item-sharded path (GpuMiner.mine_shard) all-gathers rank CSRs
                backend = comm_backend()
                make_uid = N.host_comm_unique_id if backend == "host" else N.comm_unique_id
                uid = [make_uid() if dm.rank == 0 and dm.world > 1 else b"\0" * 128]
                if dm.world > 1:
                    dist.broadcast_object_list(uid, src=0)
                self.comm = N.Comm(dm.rank, dm.world, uid[0], dm.device, backend)
        else:
            self.stream = None  # native-only single-GPU path: the miner owns its stream
            self.g = N.GpuMiner(dm.device, arena_bytes, 0)
        self.g.load_csr(tx_ptr, items, dm.n_items)
        self.n_items = dm.n_items

    def ctx(self):
        import contextlib
        return torch.cuda.stream(self.stream) if self.stream is not None else contextlib.nullcontext()

    def mine_partition(self, dm: "DistMiner", download: bool, prefetch: bool = False,
                       rule_index: bool = False):
        return self.g.mine_partition(dm.min_support, dm.max_len, download, dm.rank, dm.world,
                                     prefetch, rule_index)

    def mine_txdp(self, dm: "DistMiner", download: bool):
        return self.g.mine_txdp(self.comm, dm.n_tx, dm.min_support, dm.max_len, download,
                                dm.mfma, dm.support_tiles)

    def mine_shard(self, dm: "DistMiner", download: bool):
        """Native item-sharded call (None: the horizontal plan declined this data)."""
        if self.comm is None:
            return None
        if self.stream is not None:
            self.stream.synchronize()
        return self.g.mine_shard(self.comm, dm.n_tx, dm.min_support, dm.max_len, download,
                                 dm.support_tiles)

    def supports(self):
        c = torch.empty(self.n_items, dtype=torch.int32, device=self.dev)
        self.g.item_support(c.data_ptr())
        return c

    def select(self, host_counts: np.ndarray, n_tx: int, ms: float):
        F = self.g.select(host_counts, n_tx, ms)
        ids, counts, minsup = self.g.frequent()
        return F, ids, counts, int(minsup)

    def encode(self, F: int, ws: int):
        local = torch.zeros((F, ws), dtype=torch.int64, device=self.dev)
        self.g.encode_bitmaps(local.data_ptr(), ws, 0)
        return local

    def all_gather(self, local, world: int):
        out = torch.empty((world,) + tuple(local.shape), dtype=local.dtype, device=local.device)
        dist.all_gather_into_tensor(out, local)
        return out

    def gram(self, bm, wp: int, mfma: bool):
        F = bm.shape[0]
        gram = torch.empty((F, F), dtype=torch.int32, device=self.dev)
        self.g.pair_counts(bm.data_ptr(), wp, gram.data_ptr(), mfma)
        return gram  # stays in HBM; root_costs reduces it on the device

    def mine(self, bm, wp, dm: "DistMiner", owned, emit_level1: bool, download: bool):
        if self.stream is not None:
            self.stream.synchronize()
        return self.g.mine_bitmaps(bm.data_ptr(), wp, dm.min_support, dm.max_len, False, owned,
                                   emit_level1, download, True, dm.mfma)

    def synchronize(self):
        self.g.synchronize()


class _CpuOps:
    """The same protocol on the host (C++ kernels; gloo collectives) — CPU multi-rank tests."""

    def __init__(self, dm: "DistMiner", tx_ptr, items, arena_bytes: int):
        self.N = native.load()
        self.tx_ptr, self.items = tx_ptr, items
        self.n_items = dm.n_items
        self.rank_of = None
        self.comm = None
        if dm.mode == "tx" and dm.world > 1:  # native level loop over the shared-memory comm
            uid = [self.N.host_comm_unique_id() if dm.rank == 0 else b"\0" * 128]
            dist.broadcast_object_list(uid, src=0)
            self.comm = self.N.ShmComm(dm.rank, dm.world, uid[0])

    def mine_txdp(self, dm: "DistMiner", download: bool):
        return self.N.mine_cpu_txdp(self.tx_ptr, self.items, self.n_items, dm.n_tx,
                                    dm.min_support, dm.max_len, self.comm)

    def ctx(self):
        import contextlib
        return contextlib.nullcontext()

    def supports(self):
        c = np.bincount(self.items, minlength=self.n_items).astype(np.int32)
        return torch.from_numpy(c)

    def select(self, host_counts, n_tx, ms):
        ids, counts, rank_of, minsup = self.N.select_frequent(host_counts, n_tx, ms)
        self.rank_of = rank_of
        return len(ids), ids, counts, int(minsup)

    def encode(self, F, ws):
        bm = self.N.encode_bitmaps_cpu(self.tx_ptr, self.items, self.rank_of, F, ws)
        return torch.from_numpy(bm.view(np.int64))

    def all_gather(self, local, world):
        parts = [torch.empty_like(local) for _ in range(world)]
        dist.all_gather(parts, local)
        return torch.stack(parts)

    def gram(self, bm, wp, mfma):
        x = bm.numpy().view(np.uint64)
        bits = np.unpackbits(x.view(np.uint8), axis=1, bitorder="little").astype(np.float32)
        return (bits @ bits.T).astype(np.uint32)

    def mine(self, bm, wp, dm, owned, emit_level1, download):
        ids, counts, minsup = self.sel
        r = self.N.mine_cpu_bitmaps(np.ascontiguousarray(bm.numpy()).view(np.uint64), ids,
                                    counts, minsup, dm.max_len, owned)
        F = len(ids)
        if not emit_level1:
            r["stats"]["n_itemsets"] = int(r["stats"]["n_itemsets"]) - F
        return r

    def synchronize(self):
        pass


class DistMiner:
    """Mine one resident dataset repeatedly (the bench step / the job's mining call).

    ``backend="gpu"``: HIP kernels + RCCL (one process per MI355X).  ``backend="cpu"``: the same
    protocol with the C++ CPU kernels + gloo (used by the multi-process CPU tests)."""

    def __init__(self, tx_ptr: np.ndarray, items: np.ndarray, n_items: int, min_support: float,
                 device: int = 0, max_len: int = 0, mfma: bool = False,
                 arena_bytes: int = 0, backend: str = "gpu", force_protocol: bool = False,
                 mode: str = "auto",
                 global_n_tx: Optional[int] = None, support_tiles: int = 4):
        """``global_n_tx`` given ⇒ (tx_ptr, items) already hold only this rank's shard (tx mode;
        large datasets are generated/loaded per shard).  ``mode``: "item" (replicated bitmaps,
        item-sharded DFS), "shard" (item-sharded bitmaps, 1/N per rank: ``item_shard.py``), "replicate" (full data on every rank, device-side class partition),
        "tx" (transaction-DP, see module doc), "local" (every rank mines its OWN whole dataset
        with no collective: the dataset-parallel job / the weak-scaled bench) or "auto"."""
        self.world = dist.get_world_size() if (dist is not None and dist.is_initialized()) else 1
        self.rank = dist.get_rank() if self.world > 1 else 0
        self.n_tx = int(global_n_tx) if global_n_tx is not None else len(tx_ptr) - 1
        self.n_items = int(n_items)
        if mode == "auto":
            if global_n_tx is not None or self.n_tx >= (4 << 20):
                mode = "tx"
            elif self.world > 1 and backend == "gpu" and self.n_items <= 16384 and not mfma \
                    and not force_protocol:
                mode = "replicate"
            else:
                mode = "item"
        if mode not in ("tx", "item", "shard", "replicate", "local"):
            raise ValueError(f"unknown mode {mode!r}")
        if global_n_tx is not None and mode not in ("tx", "item", "shard"):
            raise ValueError("pre-sharded input (global_n_tx) requires mode 'tx', 'item' or 'shard'")
        self.mode = mode
        self.support_tiles = int(support_tiles)
        self.min_support = float(min_support)
        self.max_len = int(max_len)
        self.mfma = bool(mfma)
        self.device = device
        self.backend = backend
        self.force_protocol = force_protocol
        lo, hi, ts = shard_bounds(self.n_tx, self.world, self.rank)
        self.lo, self.hi, self.ts = lo, hi, ts
        if mode in ("replicate", "local"):  # every rank mines from its full (small) dataset
            sptr = np.ascontiguousarray(tx_ptr, dtype=np.int64)
            sitems = np.ascontiguousarray(items, dtype=np.int32)
        elif global_n_tx is not None:  # already this rank's shard
            sptr = np.ascontiguousarray(np.asarray(tx_ptr) - tx_ptr[0], dtype=np.int64)
            sitems = np.ascontiguousarray(items[tx_ptr[0]:tx_ptr[-1]], dtype=np.int32)
        else:
            sp = np.asarray(tx_ptr[lo:hi + 1])
            sptr = np.ascontiguousarray(sp - sp[0], dtype=np.int64)
            sitems = np.ascontiguousarray(items[sp[0]:sp[-1]], dtype=np.int32)
        ops_cls = _GpuOps if backend == "gpu" else _CpuOps
        self.ops = ops_cls(self, sptr, sitems, arena_bytes)
        self.g = getattr(self.ops, "g", None)
        self.last: Dict = {}

    def synchronize(self):
        self.ops.synchronize()

    def set_tie_rank(self, tie: np.ndarray) -> None:
        """Tie key of the device rule map's rows (``serve.index.name_tie_rank``)."""
        if self.g is not None:
            self.g.set_tie_rank(np.ascontiguousarray(tie, np.int32))

    # ------------------------------------------------------------------------------------
    def step(self, download: bool = True, reduce_count: bool = True,
             prefetch: bool = False, rule_index: bool = False) -> Dict:
        """One mining call.  Replicated mode leaves every rank's sub-trie on its own host;
        ``reduce_count=False`` skips the per-step all-reduce of the itemset count (a statistic,
        not part of the mined result: ``global_itemsets()`` reduces the last step's count once).
        ``prefetch=True`` (GPU, resident path): the next identical call is launched before this
        one is waited for, so its GPU work overlaps this call's host-side completion; the next
        ``step()`` adopts it (the steady-state loop of a serving / benchmark process)."""
        if self.mode == "replicate":
            r = self.ops.mine_partition(self, download, prefetch)
            st = dict(r["stats"])
            self._local_count = int(st["n_itemsets"])
            if reduce_count:
                st["global_itemsets"] = self.global_itemsets()
            self.last = r
            return {"stats": st, "trie": r}
        if self.mode == "shard":
            native_shard = getattr(self.ops, "mine_shard", None)
            r = native_shard(self, download) if native_shard is not None else None
            if r is not None:  # sub-trie of this rank's items (gather_trie merges them)
                st = dict(r["stats"])
                st["rounds"] = 0
                st["own_bitmap_bytes"] = st["replicated_bitmap_bytes"] = 0
                st["peak_batch_bitmap_bytes"] = st["max_batch_rows"] = 0
                st["host_phases_s"] = {k: v / 1e3 for k, v in (st.get("phases_ms") or {}).items()}
                F = int(st["n_frequent_items"])
                n_local = int(st["n_itemsets"]) - F + (F if self.rank == 0 else 0)
                tot = torch.tensor([n_local], dtype=torch.int64,
                                   device=self.ops.dev if dist.get_backend() == "nccl" else "cpu") \
                    if self.world > 1 else None
                if tot is not None:
                    dist.all_reduce(tot, op=dist.ReduceOp.SUM)
                st["n_itemsets"] = n_local
                st["global_itemsets"] = int(tot.item()) if tot is not None else n_local
                self._last_global = st["global_itemsets"]
                self.last = r
                return {"stats": st, "trie": r}
            from .item_shard import step_shard
            return step_shard(self, download)
        if self.mode == "tx":
            r = self.ops.mine_txdp(self, download and self.rank == 0)
            st = dict(r["stats"])
            st["global_itemsets"] = int(st["n_itemsets"])  # identical trie on every rank
            self._last_global = st["global_itemsets"]
            self.last = r
            return {"stats": st, "trie": r}
        if self.mode == "local" and self.backend != "gpu":  # own dataset, native CPU miner
            r = self.ops.N.mine_cpu(self.ops.tx_ptr, self.ops.items, self.n_items,
                                    self.min_support, self.max_len)
            st = dict(r["stats"])
            st["global_itemsets"] = int(st["n_itemsets"])
            self._last_global = st["global_itemsets"]
            self.last = r
            return {"stats": st, "trie": r}
        if (self.world == 1 or self.mode == "local") and self.backend == "gpu" \
                and not self.force_protocol:
            r = self.g.mine(self.min_support, self.max_len, False, download, True, self.mfma,
                            prefetch, rule_index)
            st = dict(r["stats"])
            st["global_itemsets"] = int(st["n_itemsets"])
            self._last_global = st["global_itemsets"]
            self.last = r
            return {"stats": st, "trie": r}
        return self._step_protocol(download)

    def global_itemsets(self) -> int:
        """Itemsets mined by the last step over all ranks (one all-reduce in replicated mode)."""
        if self.mode == "replicate":
            tot = torch.tensor([self._local_count], dtype=torch.int64, device=self.ops.dev)
            if self.world > 1:
                dist.all_reduce(tot, op=dist.ReduceOp.SUM)
            return int(tot.item())
        return int(self._last_global)

    def _native_comm(self):
        """This rank's native communicator for the pair ring (created once; RCCL on an nccl
        process group, the host shared-memory backend otherwise)."""
        if getattr(self, "_ncomm", None) is None:
            N = native.require_gpu()
            backend = comm_backend()
            make_uid = N.host_comm_unique_id if backend == "host" else N.comm_unique_id
            uid = [make_uid() if self.rank == 0 else b"\0" * 128]
            dist.broadcast_object_list(uid, src=0)
            self._ncomm = N.Comm(self.rank, self.world, uid[0], self.device, backend)
        return self._ncomm

    def pair_rows(self, mode: str = "reduce_scatter"):
        """Pairs-only step (``RULES_MODE=pairs``: the reference's rule map is the pair-support
        matrix): tx-sharded supports + all-reduce, selection, shard bitmaps, then one of the
        ``parallel.pairs`` strategies.  Returns (ids, row0, row1, rows) — this rank's owned rows
        of the symmetric support matrix over the frequent items ``ids`` (Eclat order)."""
        from .pairs import PairCounter
        if self.mode != "item":
            raise ValueError("pair_rows runs on the transaction-sharded protocol (mode='item')")
        ops = self.ops
        with ops.ctx():
            counts = ops.supports()
            if self.world > 1:
                dist.all_reduce(counts, op=dist.ReduceOp.SUM)
            host_counts = counts.cpu().numpy().view(np.uint32)
            F, ids, fcounts, minsup = ops.select(host_counts, self.n_tx, self.min_support)
            ops.sel = (ids, fcounts, minsup)
            X = ops.encode(F, self.ts // 64)
            comm = None
            if mode == "ring" and self.backend == "gpu" and self.world > 1:
                comm = self._native_comm()
            r0, r1, rows = PairCounter(getattr(ops, "g", None), comm).count(X, mode)
            if hasattr(rows, "cpu"):
                rows = rows.cpu()
        return ids, r0, r1, np.asarray(rows)

    def _step_protocol(self, download: bool) -> Dict:
        ops = self.ops
        t0 = time.perf_counter()
        ph: Dict[str, float] = {}
        with ops.ctx():
            # 1. transaction-DP supports + all-reduce
            counts = ops.supports()
            if self.world > 1:
                dist.all_reduce(counts, op=dist.ReduceOp.SUM)
            host_counts = counts.cpu().numpy().view(np.uint32)
            F, ids, fcounts, minsup = ops.select(host_counts, self.n_tx, self.min_support)
            ops.sel = (ids, fcounts, minsup)
            ph["supports_allreduce"] = time.perf_counter() - t0
            if F == 0:
                st = {"n_itemsets": 0, "global_itemsets": 0, "n_frequent_items": 0, "max_depth": 0}
                self._last_global = 0
                return {"stats": st, "trie": {"parent": np.zeros(0, np.int64),
                                              "item": np.zeros(0, np.int32),
                                              "count": np.zeros(0, np.uint32),
                                              "depth": np.zeros(0, np.uint8), "stats": st}}
            # 2. bitmaps of the local shard, all-gather re-shard to replicated [F][N*Ws]
            ws = self.ts // 64
            wp = ws * self.world
            local = ops.encode(F, ws)
            if self.world > 1:
                gathered = ops.all_gather(local, self.world)
                bm = gathered.permute(1, 0, 2).reshape(F, wp).contiguous()
                del gathered
            else:
                bm = local
            del local
            ph["bitmap_allgather"] = time.perf_counter() - t0
            # 3. ownership of root classes (identical on every rank, no collective)
            if self.world > 1 or self.force_protocol:
                owner = lpt_partition(root_costs(ops.gram(bm, wp, self.mfma), minsup), self.world)
                owned = (owner == self.rank).astype(np.uint8)
            else:
                owned = None
            ph["partition"] = time.perf_counter() - t0
            r = ops.mine(bm, wp, self, owned, self.rank == 0, download)
            ph["mine"] = time.perf_counter() - t0
            tot = torch.tensor([int(r["stats"]["n_itemsets"])], dtype=torch.int64,
                               device=getattr(ops, "dev", "cpu"))
            if self.world > 1:
                dist.all_reduce(tot, op=dist.ReduceOp.SUM)
            st = dict(r["stats"])
            st["global_itemsets"] = int(tot.item())
            self._last_global = st["global_itemsets"]
            st["host_phases_s"] = ph
        self.last = r
        return {"stats": st, "trie": r}


def _to_root(parts: Dict[str, np.ndarray], rank: int, world: int):
    """Every rank's 1-D arrays (same keys, same dtypes, any lengths) to rank 0 only, exactly:
    one all-gather of the lengths, then per field one ``all_to_all_single`` whose only non-empty
    splits go to rank 0 — no padding to the longest share, nothing delivered to the other ranks,
    and no extra point-to-point communicators (the collective's own group carries it).  Returns
    (lengths, {key: list of per-rank arrays}) on rank 0, (lengths, None) elsewhere."""
    dev = (torch.device("cuda", torch.cuda.current_device())
           if dist.get_backend() == "nccl" else torch.device("cpu"))
    n = len(next(iter(parts.values()))) if parts else 0
    n_local = torch.tensor([n], dtype=torch.int64, device=dev)
    sizes_t = torch.empty(world, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(sizes_t, n_local)
    sizes = [int(x) for x in sizes_t.cpu().numpy()]
    out: Dict[str, List[np.ndarray]] = {}
    for key, a in parts.items():
        a = np.ascontiguousarray(a)
        dt = getattr(torch, str(a.dtype))
        send = torch.from_numpy(a).to(dev) if n else torch.empty(0, dtype=dt, device=dev)
        recv = torch.empty(sum(sizes) if rank == 0 else 0, dtype=dt, device=dev)
        dist.all_to_all_single(recv, send,
                               output_split_sizes=sizes if rank == 0 else [0] * world,
                               input_split_sizes=[n] + [0] * (world - 1))
        if rank == 0:
            h = recv.cpu().numpy()
            offs = np.concatenate([[0], np.cumsum(sizes)])
            out[key] = [h[offs[q]:offs[q + 1]] for q in range(world)]
    return sizes, (out if rank == 0 else None)


def gather_arrays(arrs: Dict[str, np.ndarray], rank: int, world: int
                  ) -> Optional[Dict[str, np.ndarray]]:
    """Concatenate equally-keyed 1-D arrays of every rank on rank 0 (rank order): exact-size
    transfers to rank 0 only (``_to_root``)."""
    if world == 1:
        return {k: np.asarray(v) for k, v in arrs.items()}
    _, got = _to_root(arrs, rank, world)
    if rank != 0:
        return None
    return {k: np.concatenate(v) for k, v in got.items()}


def gather_trie(r: Dict, rank: int, world: int, n_frequent: int) -> Optional[Dict[str, np.ndarray]]:
    """Concatenate per-rank sub-tries on rank 0 (level-1 nodes 0..F-1 are shared; every rank's
    local ids >= F are rebased).

    Transport: tensor collectives on the process group's device (HBM for RCCL, host for gloo),
    exact sizes to rank 0 only (``_to_root``: one all-gather of the sizes, one all_to_all_single
    per field) — the other ranks receive nothing, and no share is padded to the largest."""
    fields = ("parent", "item", "count", "depth")
    if world == 1:
        return {k: np.asarray(r[k]) for k in fields}
    F = n_frequent
    mine = {"parent": np.asarray(r["parent"], np.int64)[F:], "item": np.asarray(r["item"], np.int32)[F:],
            "count": np.asarray(r["count"]).astype(np.uint32).view(np.int32)[F:],
            "depth": np.asarray(r["depth"], np.uint8)[F:]}
    sizes, parts = _to_root(mine, rank, world)
    if rank != 0:
        return None
    head = {k: np.asarray(r[k])[:F] for k in fields}
    out = {"parent": [head["parent"].astype(np.int64)], "item": [head["item"].astype(np.int32)],
           "count": [head["count"].astype(np.uint32)], "depth": [head["depth"].astype(np.uint8)]}
    base = F
    for q in range(world):
        n = int(sizes[q])
        if n == 0:
            continue
        par = parts["parent"][q].copy()
        loc = par >= F
        par[loc] += base - F
        out["parent"].append(par)
        out["item"].append(parts["item"][q])
        out["count"].append(parts["count"][q].view(np.uint32))
        out["depth"].append(parts["depth"][q])
        base += n
    return {k: np.concatenate(v) for k, v in out.items()}
