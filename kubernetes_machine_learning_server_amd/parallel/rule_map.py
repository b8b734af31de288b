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
        self.s = self.stream.cuda_stream
        self.g = N.GpuMiner(rm.device, 1 << 30, self.s)
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

    def supports(self, rm: "DistRuleMap"):
        """Global per-item supports: the shard histogram, all-reduced — left on the device (the
        selection reads them there; a checkpoint copies them out)."""
        with torch.cuda.stream(self.stream):
            cnt = self.buf("cnt", (rm.n_items,), torch.int32)
            cnt.zero_()
            self.g.item_support(cnt.data_ptr())
            if self.comm is not None:
                self.comm.all_reduce(cnt.data_ptr(), cnt.data_ptr(), rm.n_items, "u32", False,
                                     self.s)
                self.comm.wait_stream(self.s)
            return cnt

    def counts_to_host(self, counts) -> np.ndarray:
        self.stream.synchronize()
        return counts.cpu().numpy().view(np.uint32).copy()

    def select(self, rm: "DistRuleMap", counts):
        """The selection on the device (``select_device``): no 4 MB count / rank-table copies and
        no host scan of the 1M-item vocabulary per step.  Counts restored from a checkpoint are
        uploaded and take the same path, so a resumed step ranks the items identically."""
        if isinstance(counts, np.ndarray):
            with torch.cuda.stream(self.stream):
                cnt = self.buf("cnt", (rm.n_items,), torch.int32)
                cnt.copy_(torch.from_numpy(np.ascontiguousarray(counts, np.uint32).view(np.int32)))
            counts = cnt
        with torch.cuda.stream(self.stream):
            F = self.g.select_device(counts.data_ptr(), rm.n_tx, rm.min_support)
        ids, fcounts, minsup = self.g.frequent()
        return F, np.asarray(ids), np.asarray(fcounts), int(minsup)

    def gram_rows(self, rm: "DistRuleMap", F: int):
        """This rank's rows of the summed, mirrored gram (device tensor [per][F]).

        The shard's gram is counted horizontally from its CSR (``cooc.hip``: every co-occurring
        frequent pair once; no bitmaps at all) when the cost model prefers it — at config 5
        (~7 frequent items per transaction) by orders of magnitude — else through the shard's
        tid-bitmaps and the MFMA bit-GEMM."""
        per, _, _ = row_block(F, rm.world, rm.rank)
        with torch.cuda.stream(self.stream):
            gram = self.buf("gram", (per * rm.world, max(F, 1)), torch.int32)
            if per * rm.world > F:
                gram[F:] = 0
            self.method = "none"
            if F:
                # the cost model from the supports (no statistics pass over the CSR); a
                # transaction past the count's entry buffer sends the call to the bit-GEMM
                if self.g.cooc_likely() and self.g.pair_counts_csr_direct(gram.data_ptr(), F):
                    self.method = "cooc"
                    self.held.pop("bm", None)
                else:
                    self.method = "gram"
                    bm = self.buf("bm", (max(F, 1), self.Ws), torch.int64)
                    if self.Ws > self.used:
                        bm[:, self.used:] = 0
                    self.g.encode_bitmaps(bm.data_ptr(), self.Ws, 0)
                    self.g.pair_counts(bm.data_ptr(), self.Ws, gram.data_ptr(), True)
                self.g.gram_mirror(gram.data_ptr(), F, F)
            if self.comm is None:
                return gram
            rows = self.buf("rows", (per, max(F, 1)), torch.int32)
            self.comm.reduce_scatter(gram.data_ptr(), rows.data_ptr(), per * max(F, 1), "u32",
                                     False, self.s)
            self.comm.wait_stream(self.s)
            return rows

    def rows_to_host(self, rows) -> np.ndarray:
        self.stream.synchronize()
        return rows.cpu().numpy()

    def rows_from_host(self, rm: "DistRuleMap", a: np.ndarray, F: int):
        with torch.cuda.stream(self.stream):
            t = self.buf("rows", tuple(a.shape), torch.int32)
            t.copy_(torch.from_numpy(np.ascontiguousarray(a)))
            return t

    def rows_csr(self, rm: "DistRuleMap", rows, F: int, r0: int, nrows: int, minsup: int):
        self.stream.synchronize()
        return self.g.rule_map_rows(rows.data_ptr(), max(F, 1), r0, nrows, minsup)

    def release(self):
        self.held.clear()


def _deltas_ms(ph: Dict[str, float]) -> Dict[str, float]:
    """Cumulative phase-end marks (s) -> each phase's own duration (ms)."""
    out, prev = {}, 0.0
    for k, v in ph.items():
        out[k] = round((v - prev) * 1e3, 3)
        prev = v
    return out


class _Cpu:
    def __init__(self, rm: "DistRuleMap", tx_ptr, items):
        self.N = native.load()
        self.tx_ptr = np.ascontiguousarray(tx_ptr, np.int64)
        self.items = np.ascontiguousarray(items, np.int32)
        self.comm = None
        self.tie = None
        self.rank_of = None
        if rm.world > 1:
            uid = [self.N.host_comm_unique_id() if rm.rank == 0 else b"\0" * 128]
            dist.broadcast_object_list(uid, src=0)
            self.comm = self.N.ShmComm(rm.rank, rm.world, uid[0])

    def set_tie_rank(self, tie):
        self.tie = np.asarray(tie, np.int64)

    def counts_to_host(self, counts) -> np.ndarray:
        return np.asarray(counts, np.uint32)

    def supports(self, rm: "DistRuleMap") -> np.ndarray:
        cnt = np.bincount(self.items, minlength=rm.n_items).astype(np.uint32)
        if self.comm is not None:
            self.comm.all_reduce(cnt, False)
        return cnt

    def select(self, rm: "DistRuleMap", counts: np.ndarray):
        ids, fcounts, rank_of, minsup = self.N.select_frequent(counts, rm.n_tx, rm.min_support)
        self.rank_of = rank_of
        return len(ids), np.asarray(ids), np.asarray(fcounts), int(minsup)

    def gram_rows(self, rm: "DistRuleMap", F: int):
        per, _, _ = row_block(F, rm.world, rm.rank)
        W = (len(self.tx_ptr) - 1 + 63) // 64
        bm = self.N.encode_bitmaps_cpu(self.tx_ptr, self.items, self.rank_of, F, W)
        bits = np.unpackbits(np.ascontiguousarray(bm).view(np.uint8).reshape(F, -1), axis=1,
                             bitorder="little").astype(np.float32)
        gram = np.zeros((per * rm.world, max(F, 1)), np.uint32)
        gram[:F, :F] = np.rint(bits @ bits.T).astype(np.uint32)  # full symmetric
        if self.comm is None:
            return gram
        return self.comm.reduce_scatter(gram.reshape(-1), False).reshape(per, -1)

    def rows_to_host(self, rows) -> np.ndarray:
        return np.asarray(rows)

    def rows_from_host(self, rm: "DistRuleMap", a: np.ndarray, F: int):
        return np.asarray(a, np.uint32)

    def rows_csr(self, rm: "DistRuleMap", rows, F: int, r0: int, nrows: int, minsup: int):
        ids = self.ids
        return rows_csr_host(np.asarray(rows)[:nrows, :F], r0, ids, minsup, self.tie)

    def release(self):
        pass


class DistRuleMap:
    """The rule map of one dataset whose transactions are sharded over the ranks.

    ``tx_ptr``/``items``: this rank's shard (global transaction count ``global_n_tx``).
    ``step()`` returns the item-id CSR on rank 0 (``row_ptr``/``cons``/``count``, plus the
    frequent ids/counts and per-phase times) and ``None`` elsewhere.

    Phase checkpoints (``ck`` = a ``utils.checkpoint.PhaseCheckpoint``): the global
    supports (rank 0), every rank's reduce-scattered gram rows (the seconds of MFMA work at HBM
    scale) and every rank's CSR rows.  A restarted call resumes after the last phase that EVERY
    rank has (one MIN all-reduce of the ranks' phase levels); the frequent order is a pure
    function of the supports, so it is recomputed, not stored."""

    def __init__(self, tx_ptr, items, n_items: int, global_n_tx: int, min_support: float,
                 device: int = 0, backend: str = "gpu", comm_backend: Optional[str] = None,
                 ck=None):
        self.world = dist.get_world_size() if (dist is not None and dist.is_initialized()) else 1
        self.rank = dist.get_rank() if self.world > 1 else 0
        self.n_items, self.n_tx = int(n_items), int(global_n_tx)
        self.min_support = float(min_support)
        self.device = device
        self.ck = ck
        self.comm_backend = comm_backend or os.environ.get("KMLS_COMM") or (
            "rccl" if self.world > 1 and dist.get_backend() == "nccl" else "host")
        self.ops = (_Gpu if backend == "gpu" else _Cpu)(self, tx_ptr, items)

    def set_tie_rank(self, tie: np.ndarray) -> None:
        self.ops.set_tie_rank(tie)

    def _phase(self, name: str) -> str:
        return f"rulemap_{name}_r{self.rank}of{self.world}"

    def _resume_level(self) -> int:
        """0 nothing, 1 supports, 2 gram rows, 3 CSR rows — the minimum over the ranks."""
        ck = self.ck
        if ck is None or not ck.enabled:
            return 0
        lvl = 0
        if ck.has("rulemap_supports"):
            lvl = 1
            if ck.has(self._phase("rows")):
                lvl = 2
                if ck.has(self._phase("csr")):
                    lvl = 3
        if self.world > 1:
            t = torch.tensor([lvl], dtype=torch.int64,
                             device="cuda" if dist.get_backend() == "nccl" else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            lvl = int(t.item())
        return lvl

    def step(self) -> Optional[Dict]:
        from .dist_miner import gather_arrays
        ph: Dict[str, float] = {}
        t0 = time.perf_counter()
        ck, ops = self.ck, self.ops
        lvl = self._resume_level()
        if lvl >= 1:
            counts = ck.load("rulemap_supports")["counts"]
        else:
            counts = ops.supports(self)
            if ck is not None and ck.enabled and self.rank == 0:
                ck.save("rulemap_supports", counts=ops.counts_to_host(counts))
        ph["supports_allreduce"] = time.perf_counter() - t0
        F, ids, fcounts, minsup = ops.select(self, counts)
        ops.ids = ids
        per, r0, nrows = row_block(F, self.world, self.rank)
        loc = None
        if lvl >= 3:
            z = ck.load(self._phase("csr"))
            loc = {"row_ptr": z["row_ptr"], "cons": z["cons"], "count": z["count"],
                   "status": int(z["status"])}
        else:
            if lvl >= 2:
                rows = ops.rows_from_host(self, ck.load(self._phase("rows"))["rows"], F)
            else:
                rows = ops.gram_rows(self, F)
                if ck is not None and ck.enabled:
                    ck.save(self._phase("rows"), rows=ops.rows_to_host(rows))
            if hasattr(ops, "stream"):  # the phase's device work ends inside the phase
                ops.stream.synchronize()
            ph["encode_gram_reduce_scatter"] = time.perf_counter() - t0
            loc = ops.rows_csr(self, rows, F, r0, nrows, minsup)
            if ck is not None and ck.enabled:
                ck.save(self._phase("csr"), row_ptr=np.asarray(loc["row_ptr"]),
                        cons=np.asarray(loc["cons"]), count=np.asarray(loc["count"]),
                        status=np.int64(loc.get("status", 0)))
        ph["rows_csr"] = time.perf_counter() - t0
        if os.environ.get("KMLS_FAULT") == "rulemap_after_csr":
            raise RuntimeError("injected fault at rulemap_after_csr")
        lens = np.diff(np.asarray(loc["row_ptr"], np.int64))
        # every rank's rule_map_rows status rides along (bit 1: fill overflow, bit 2: a row
        # sorted past kSortBig): a bad row block on ANY rank fails the assembled map
        got_l = gather_arrays({"lens": lens.astype(np.int64)}, self.rank, self.world)
        got_s = gather_arrays({"status": np.array([int(loc.get("status", 0))], np.int64)},
                              self.rank, self.world)
        got_e = gather_arrays({"cons": np.asarray(loc["cons"], np.int32),
                               "count": np.asarray(loc["count"], np.uint32).view(np.int32)},
                              self.rank, self.world)
        ph["gather"] = time.perf_counter() - t0
        if self.rank != 0:
            return None
        status = int(np.bitwise_or.reduce(np.asarray(got_s["status"], np.int64)))
        if status:
            raise RuntimeError(f"DistRuleMap: rule_map_rows status {status} on some rank "
                               "(1: fill overflow, 2: unsorted long row)")
        out = assemble_by_id(ids, got_l["lens"][:F], got_e["cons"],
                             got_e["count"].view(np.uint32), self.n_items)
        ph["assemble"] = time.perf_counter() - t0
        out.update(ids=ids, fcounts=fcounts, minsup=minsup, n_frequent_items=F,
                   status=status, resumed_from_phase=lvl,
                   level2_method=getattr(ops, "method", "gram"),
                   # wall time of each phase (device work of a phase waited for at its end)
                   phases_ms=_deltas_ms(ph))
        return out

    def release(self) -> None:
        self.ops.release()
