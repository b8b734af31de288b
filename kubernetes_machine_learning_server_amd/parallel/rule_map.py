"""BASELINE config 5 across ranks: the deployed artifact (the pair rule map) at HBM scale, one
process per GPU.

The reference builds its rule map on one host (``machine-learning/main.py:282-304``: for every
frequent itemset S and song a in S, rec[a][b] = max(rec[a][b], support(S)), which is the
pair-support matrix).  At 100M transactions x 1M items the bitmap of the >10k frequent
items is ~185 GB, so here every rank owns a transaction shard and the F x F gram is split by
rows:

1. supports of the rank's shard (HIP histogram) -> ``all_reduce`` (native communicator: RCCL
   over xGMI, or host shared memory) -> the same frequent-item selection on every rank;
2. tid-bitmaps of the shard ([F][T/N/64] words, ~185/N GB) -> the shard's MFMA gram (upper
   triangle), mirrored to full symmetric rows (``gram_mirror``);
3. ``reduce_scatter`` of contiguous row blocks: rank g receives rows [g*Fp/N, (g+1)*Fp/N) of the
   summed gram, all F columns (one large collective: (N-1)/N of a 0.9 GB gram per rank,
   ring-bound on the point-to-point links);
4. the CSR of its rows (``rule_map_rows``: survivors, count-desc/tie-asc sort, consequents as
   item ids) — each rank builds 1/N of the map;
5. a gather of the row blocks to rank 0, which re-indexes them by item id: the same CSR
   (row_ptr / cons / count) as the single-GPU ``rule_map_from_gram``, hence the same
   ``rules.idx`` bytes.

``backend="cpu"`` runs the identical protocol with numpy/C++ host kernels and the host
shared-memory communicator (the multi-process CPU test tier).
"""
from __future__ import annotations

import os
import time
from typing import Dict, Optional

import numpy as np

from ..ops import native

try:
    import torch
    import torch.distributed as dist
except Exception:  # pragma: no cover
    torch = None
    dist = None


def row_block(F: int, world: int, rank: int):
    """(per, r0, nrows): rows per rank (F padded to a multiple of world) and this rank's rows."""
    per = -(-max(F, 1) // world)
    r0 = min(F, rank * per)
    return per, r0, max(0, min(F, r0 + per) - r0)


def assemble_by_id(ids: np.ndarray, lens: np.ndarray, cons: np.ndarray, cnt: np.ndarray,
                   n_items: int) -> Dict[str, np.ndarray]:
    """Rows in frequent-rank order (row r = item ids[r]) -> the CSR indexed by item id."""
    ids = np.asarray(ids, np.int64)
    lens = np.asarray(lens, np.int64)
    start = np.zeros(len(lens), np.int64)
    if len(lens) > 1:
        np.cumsum(lens[:-1], out=start[1:])
    by_id = np.zeros(n_items + 1, np.int64)
    by_id[ids] = lens
    row_ptr = np.zeros(n_items + 1, np.int64)
    np.cumsum(by_id[:n_items], out=row_ptr[1:])
    order = np.argsort(ids, kind="stable")
    nnz = int(lens.sum())
    src = np.arange(nnz, dtype=np.int64) + np.repeat(start[order] - row_ptr[ids[order]],
                                                     lens[order])
    return {"row_ptr": row_ptr, "cons": np.asarray(cons, np.int32)[src],
            "count": np.asarray(cnt, np.uint32)[src], "nnz": nnz}


def rows_csr_host(rows: np.ndarray, r0: int, ids: np.ndarray, minsup: int,
                  tie: Optional[np.ndarray] = None) -> Dict[str, np.ndarray]:
    """Host reference of ``GpuMiner.rule_map_rows``: CSR of a full-row block (rows r0.., all F
    columns), entries j != own row with count >= minsup, ordered count desc, tie key asc."""
    nrows, F = rows.shape
    keep = rows >= minsup
    if nrows:
        keep[np.arange(nrows), np.arange(r0, r0 + nrows)] = False
    rr, jj = np.nonzero(keep)
    c = rows[rr, jj].astype(np.int64)
    cons = np.asarray(ids, np.int64)[jj]
    t = cons if tie is None else np.asarray(tie, np.int64)[cons]
    o = np.lexsort((t, -c, rr))
    lens = np.bincount(rr, minlength=nrows).astype(np.int64)
    row_ptr = np.zeros(nrows + 1, np.int64)
    np.cumsum(lens, out=row_ptr[1:])
    return {"row_ptr": row_ptr, "cons": cons[o].astype(np.int32),
            "count": c[o].astype(np.uint32), "nnz": int(len(o)), "status": 0}


class _Gpu:
    def __init__(self, rm: "DistRuleMap", tx_ptr, items):
        N = native.require_gpu()
        self.N = N
        torch.cuda.set_device(rm.device)
        self.dev = torch.device("cuda", rm.device)
        # torch fills, the native kernels and the communicator all run on ONE stream
        self.stream = torch.cuda.Stream(device=rm.device)
        self.g = N.GpuMiner(rm.device, 1 << 30, self.stream.cuda_stream)
        self.g.load_csr(tx_ptr, items, rm.n_items)
        self.comm = None
        if rm.world > 1:
            backend = rm.comm_backend
            make = N.host_comm_unique_id if backend == "host" else N.comm_unique_id
            uid = [make() if rm.rank == 0 else b"\0" * 128]
            dist.broadcast_object_list(uid, src=0)
            self.comm = N.Comm(rm.rank, rm.world, uid[0], rm.device, backend)
        self.held: Dict[str, "torch.Tensor"] = {}  # HBM buffers kept across calls
        self.Ws = self.g.words_local()
        self.used = (len(tx_ptr) - 1 + 63) // 64

    def buf(self, name, shape, dtype):
        t = self.held.get(name)
        if t is None or tuple(t.shape) != tuple(shape):
            self.held.pop(name, None)
            t = self.held[name] = torch.empty(shape, dtype=dtype, device=self.dev)
        return t

    def set_tie_rank(self, tie):
        self.g.set_tie_rank(np.ascontiguousarray(tie, np.int32))

    def step(self, rm: "DistRuleMap", ph: Dict[str, float]):
        s = self.stream.cuda_stream
        t0 = time.perf_counter()
        with torch.cuda.stream(self.stream):
            cnt = self.buf("cnt", (rm.n_items,), torch.int32)
            cnt.zero_()
            self.g.item_support(cnt.data_ptr())
            if self.comm is not None:
                self.comm.all_reduce(cnt.data_ptr(), cnt.data_ptr(), rm.n_items, "u32", False, s)
                self.comm.wait_stream(s)
            host = cnt.cpu().numpy().view(np.uint32)
            ph["supports_allreduce"] = time.perf_counter() - t0
            F = self.g.select(host, rm.n_tx, rm.min_support)
            ids, fcounts, minsup = self.g.frequent()
            per, r0, nrows = row_block(F, rm.world, rm.rank)
            bm = self.buf("bm", (max(F, 1), self.Ws), torch.int64)
            if self.Ws > self.used:
                bm[:, self.used:] = 0
            if F:
                self.g.encode_bitmaps(bm.data_ptr(), self.Ws, 0)
            gram = self.buf("gram", (per * rm.world, max(F, 1)), torch.int32)
            if per * rm.world > F:
                gram[F:] = 0
            if F:
                self.g.pair_counts(bm.data_ptr(), self.Ws, gram.data_ptr(), True)
                self.g.gram_mirror(gram.data_ptr(), F, F)
            self.stream.synchronize()
            ph["encode_gram"] = time.perf_counter() - t0
            if self.comm is not None:
                rows = self.buf("rows", (per, max(F, 1)), torch.int32)
                self.comm.reduce_scatter(gram.data_ptr(), rows.data_ptr(), per * max(F, 1), "u32",
                                         False, s)
                self.comm.wait_stream(s)
            else:
                rows = gram
            self.stream.synchronize()
            ph["reduce_scatter"] = time.perf_counter() - t0
            loc = self.g.rule_map_rows(rows.data_ptr(), max(F, 1), r0, nrows, int(minsup))
            ph["rows_csr"] = time.perf_counter() - t0
        return F, np.asarray(ids), np.asarray(fcounts), int(minsup), loc

    def release(self):
        self.held.clear()


class _Cpu:
    def __init__(self, rm: "DistRuleMap", tx_ptr, items):
        self.N = native.load()
        self.tx_ptr = np.ascontiguousarray(tx_ptr, np.int64)
        self.items = np.ascontiguousarray(items, np.int32)
        self.comm = None
        self.tie = None
        if rm.world > 1:
            uid = [self.N.host_comm_unique_id() if rm.rank == 0 else b"\0" * 128]
            dist.broadcast_object_list(uid, src=0)
            self.comm = self.N.ShmComm(rm.rank, rm.world, uid[0])

    def set_tie_rank(self, tie):
        self.tie = np.asarray(tie, np.int64)

    def step(self, rm: "DistRuleMap", ph: Dict[str, float]):
        t0 = time.perf_counter()
        cnt = np.bincount(self.items, minlength=rm.n_items).astype(np.uint32)
        if self.comm is not None:
            self.comm.all_reduce(cnt, False)
        ph["supports_allreduce"] = time.perf_counter() - t0
        ids, fcounts, rank_of, minsup = self.N.select_frequent(cnt, rm.n_tx, rm.min_support)
        F = len(ids)
        per, r0, nrows = row_block(F, rm.world, rm.rank)
        W = (len(self.tx_ptr) - 1 + 63) // 64
        bm = self.N.encode_bitmaps_cpu(self.tx_ptr, self.items, rank_of, F, W)
        bits = np.unpackbits(np.ascontiguousarray(bm).view(np.uint8).reshape(F, -1), axis=1,
                             bitorder="little").astype(np.float32)
        gram = np.zeros((per * rm.world, max(F, 1)), np.uint32)
        gram[:F, :F] = np.rint(bits @ bits.T).astype(np.uint32)  # full symmetric
        ph["encode_gram"] = time.perf_counter() - t0
        rows = (self.comm.reduce_scatter(gram.reshape(-1), False).reshape(per, -1)
                if self.comm is not None else gram)
        ph["reduce_scatter"] = time.perf_counter() - t0
        loc = rows_csr_host(rows[:nrows, :F], r0, ids, int(minsup), self.tie)
        ph["rows_csr"] = time.perf_counter() - t0
        return F, np.asarray(ids), np.asarray(fcounts), int(minsup), loc

    def release(self):
        pass


class DistRuleMap:
    """The rule map of one dataset whose transactions are sharded over the ranks.

    ``tx_ptr``/``items``: this rank's shard (global transaction count ``global_n_tx``).
    ``step()`` returns the item-id CSR on rank 0 (``row_ptr``/``cons``/``count``, plus the
    frequent ids/counts and per-phase times) and ``None`` elsewhere."""

    def __init__(self, tx_ptr, items, n_items: int, global_n_tx: int, min_support: float,
                 device: int = 0, backend: str = "gpu", comm_backend: Optional[str] = None):
        self.world = dist.get_world_size() if (dist is not None and dist.is_initialized()) else 1
        self.rank = dist.get_rank() if self.world > 1 else 0
        self.n_items, self.n_tx = int(n_items), int(global_n_tx)
        self.min_support = float(min_support)
        self.device = device
        self.comm_backend = comm_backend or os.environ.get("KMLS_COMM") or (
            "rccl" if self.world > 1 and dist.get_backend() == "nccl" else "host")
        self.ops = (_Gpu if backend == "gpu" else _Cpu)(self, tx_ptr, items)

    def set_tie_rank(self, tie: np.ndarray) -> None:
        self.ops.set_tie_rank(tie)

    def step(self) -> Optional[Dict]:
        from .dist_miner import gather_arrays
        ph: Dict[str, float] = {}
        t0 = time.perf_counter()
        F, ids, fcounts, minsup, loc = self.ops.step(self, ph)
        lens = np.diff(np.asarray(loc["row_ptr"], np.int64))
        parts = {"lens": lens.astype(np.int64)}
        got_l = gather_arrays(parts, self.rank, self.world)
        got_e = gather_arrays({"cons": np.asarray(loc["cons"], np.int32),
                               "count": np.asarray(loc["count"], np.uint32).view(np.int32)},
                              self.rank, self.world)
        ph["gather"] = time.perf_counter() - t0
        if self.rank != 0:
            return None
        out = assemble_by_id(ids, got_l["lens"][:F], got_e["cons"],
                             got_e["count"].view(np.uint32), self.n_items)
        ph["assemble"] = time.perf_counter() - t0
        out.update(ids=ids, fcounts=fcounts, minsup=minsup, n_frequent_items=F,
                   status=int(loc.get("status", 0)),
                   phases_ms={k: round(v * 1e3, 3) for k, v in ph.items()})
        return out

    def release(self) -> None:
        self.ops.release()
