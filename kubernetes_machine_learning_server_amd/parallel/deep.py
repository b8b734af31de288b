"""Count-only full FP-Growth mining of ONE dataset split over the GPUs of a node.

The reference mines every frequent itemset of every size (``machine-learning/main.py:272``) and
sweeps min_support downwards (``main.py:450-473``).  At the BASELINE config-2 family (ds1 at
0.01-0.02) the output is 1e9-1e10 itemsets: every itemset and its support is computed, the
per-size counts and the content digest (``kmls/digest.hpp``, equal to the digest of the full
trie) are kept, nothing is materialised (``GpuMiner.mine_deep``, ``csrc/kernels/deep.hip``).

Split over ranks (strong scaling): every rank builds the same level-2 classes on its own GPU
(deterministic), rank r mines the level-3 tasks t with t % world == r, and the per-size counts
and digest sums are all-reduced (the digest xors all-gathered), so every rank ends with the
result of the whole problem.  The combine runs through one of:

* ``"rccl"``  — the native communicator (``csrc/host/comm_rccl.cpp``: RCCL over xGMI, issued on
  the miner's stream inside ``mine_deep``);
* ``"host"``  — the native host shared-memory communicator (ranks sharing one GPU, CPU tests);
* ``"torch"`` — ``torch.distributed`` on the job's process group (RCCL on an ``nccl`` group,
  gloo otherwise): one 66-word all-reduce + one all-gather per call, after ``mine_deep``
  returned the rank's partial.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional

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

    def _combine_torch(self, d: Dict) -> Dict:
        return allreduce_partial(d, self.world, self.device)

    def synchronize(self) -> None:
        self.g.synchronize()
