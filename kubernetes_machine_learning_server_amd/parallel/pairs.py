"""Distributed level-2 pair counting — the SURVEY §2.E parallelism rows for the pair-support matrix.

The reference's deployed rule map is exactly the pair-support matrix (SURVEY §0;
``machine-learning/main.py:282-296``), so ``RULES_MODE=pairs`` only needs G = XᵀX over the
transactions.  With transactions sharded over N ranks (rank r holds X_r = the [F][Ws] tid-bitmap
words of its shard for every frequent item), four strategies produce G:

* ``allreduce``      — DP: each rank computes its partial G_r = X_r·X_rᵀ, one all-reduce.  Every
  rank ends with all of G (F² words on the wire, per-link bound on an xGMI ring).
* ``reduce_scatter`` — DP + item ownership: partial G_r, then ``reduce_scatter`` of row blocks,
  so rank r receives only its rows S_r (1/N of the bytes of an all-reduce's result).
* ``alltoall``       — Ulysses analog: the partial row blocks are exchanged with one
  ``all_to_all`` (tx-sharded partials → item-sharded sums) and summed locally.
* ``ring``           — context-parallel / ring-attention analog: rank r keeps its owned rows
  resident ("Q stays") while the transaction blocks X_j rotate around the ring ("KV rotates")
  with send/recv; step k computes G[S_r, :] += X_j[S_r]·X_jᵀ on the matrix engine of rank r
  while X_j travels on to the next rank.  Peak memory is two blocks instead of N.  With a native
  communicator the whole pass runs in C++ (``GpuMiner.ring_pair_rows``: RCCL / host sendrecv on
  a side stream, events ordering it against the bit-GEMM on the miner's stream).

Every strategy returns the same thing: ``(row0, row1, rows)`` with ``rows[i][j]`` = support of
items (row0+i, j) — the symmetric count matrix, diagonal = item supports.  GPU ranks use the
HIP rectangular bit-GEMM (``GpuMiner.bitgemm_rect``) on the miner's stream, with RCCL ops
ordered against it; CPU ranks (tests) use numpy + gloo.
"""
from __future__ import annotations

from typing import Tuple

import numpy as np

try:
    import torch
    import torch.distributed as dist
except Exception:  # pragma: no cover
    torch = None
    dist = None

MODES = ("allreduce", "reduce_scatter", "alltoall", "ring")


def row_block(F: int, world: int, rank: int) -> Tuple[int, int, int]:
    """(row0, row1, Fb): rank's owned rows of G; Fb = padded block height."""
    fb = -(-F // world) if world > 0 else F
    r0 = min(F, rank * fb)
    return r0, min(F, r0 + fb), fb


def _cpu_rect(a: "torch.Tensor", b: "torch.Tensor") -> "torch.Tensor":
    """popcount(a_i & b_j) for int64 bitmap rows (CPU: unpack + fp64 matmul, exact)."""
    def bits(x):
        u = np.ascontiguousarray(x.numpy()).view(np.uint8)
        return np.unpackbits(u, axis=1, bitorder="little").astype(np.float64)
    return torch.from_numpy((bits(a) @ bits(b).T).astype(np.int64))


class PairCounter:
    """Runs one strategy on a rank.  ``miner``: the rank's ``_native.GpuMiner`` (its stream must
    be torch's current stream — see DistMiner's protocol ops) or None for the CPU backend."""

    def __init__(self, miner=None, comm=None):
        self.g = miner
        self.comm = comm  # native Comm (RCCL / host): the ring runs in C++ on a side stream

    def _rect(self, a, b, out=None):
        """out[i][j] += popcount(a_i & b_j); returns out."""
        if self.g is None:
            r = _cpu_rect(a, b)
            return r if out is None else out.add_(r)
        if out is None:
            out = torch.zeros((a.shape[0], b.shape[0]), dtype=torch.int32, device=a.device)
        if a.shape[0] and b.shape[0]:
            self.g.bitgemm_rect(a.data_ptr(), a.shape[0], b.data_ptr(), b.shape[0], a.shape[1],
                                out.data_ptr(), out.shape[1])
        return out

    def count(self, X: "torch.Tensor", mode: str = "reduce_scatter"):
        """X: this rank's [F][Ws] int64 bitmap words (identical F and Ws on every rank)."""
        if mode not in MODES:
            raise ValueError(f"unknown pair mode {mode!r}; choose from {MODES}")
        world = dist.get_world_size() if (dist is not None and dist.is_initialized()) else 1
        rank = dist.get_rank() if world > 1 else 0
        F = X.shape[0]
        r0, r1, fb = row_block(F, world, rank)
        if world == 1:
            return 0, F, self._rect(X, X)
        if mode == "allreduce":
            G = self._rect(X, X)
            dist.all_reduce(G)
            return r0, r1, G[r0:r1]
        if mode in ("reduce_scatter", "alltoall"):
            pad = torch.zeros((world * fb, F), dtype=torch.int32 if self.g is not None else torch.int64,
                              device=X.device)
            self._rect(X, X, pad[:F])
            if mode == "reduce_scatter":
                out = torch.empty((fb, F), dtype=pad.dtype, device=X.device)
                dist.reduce_scatter_tensor(out, pad)
            else:
                recv = torch.empty_like(pad)
                dist.all_to_all_single(recv, pad)  # block h of every rank → rank h
                out = recv.view(world, fb, F).sum(dim=0, dtype=pad.dtype)
            return r0, r1, out[: r1 - r0]
        # ring: owned rows stay, transaction blocks rotate
        acc = torch.zeros((fb, F), dtype=torch.int32 if self.g is not None else torch.int64,
                          device=X.device)
        if self.g is not None and self.comm is not None:
            # native (GpuMiner::ring_pair_rows): sendrecv of block k+1 on the communicator's
            # stream overlapped with block k's bit-GEMM on the miner's stream
            X = X.contiguous()
            self.g.ring_pair_rows(self.comm, X.data_ptr(), F, X.shape[1], acc.data_ptr(), F)
            return r0, r1, acc[: r1 - r0]
        cur = X.contiguous()
        nxt = torch.empty_like(cur)
        for k in range(world):
            reqs = []
            if k < world - 1:
                ops = [dist.P2POp(dist.isend, cur, (rank + 1) % world),
                       dist.P2POp(dist.irecv, nxt, (rank - 1) % world)]
                reqs = dist.batch_isend_irecv(ops)
            self._rect(cur[r0:r1], cur, acc[: r1 - r0])  # overlaps the transfer above
            for q in reqs:
                q.wait()
            cur, nxt = nxt, cur
        return r0, r1, acc[: r1 - r0]
