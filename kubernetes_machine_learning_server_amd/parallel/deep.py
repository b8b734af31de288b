"""Count-only full FP-Growth mining of ONE dataset split over the GPUs of a node.

The reference mines every frequent itemset of every size (``machine-learning/main.py:272``) and
sweeps min_support downwards (``main.py:450-473``).  At the BASELINE config-2 family (ds1 at
0.01-0.02) the output is 1e9-1e10 itemsets: every itemset and its support is computed, the
per-size counts and the content digest (``kmls/digest.hpp``, equal to the digest of the full
trie) are kept, nothing is materialised (``GpuMiner.mine_deep``, ``csrc/kernels/deep.hip``).

Split over ranks (strong scaling): every rank builds the same level-2 classes on its own GPU
(deterministic), rank r mines the level-3 tasks t with t % world == r, and the per-size counts
and digest sums are all-reduced (the digest xors all-gathered) through the native communicator
(``csrc/host/comm_rccl.cpp``: RCCL over xGMI on an nccl process group, the host shared-memory
backend otherwise), so every rank ends with the result of the whole problem.
"""
from __future__ import annotations

import os
from typing import Dict, Optional

from ..ops import native

try:
    import torch
    import torch.distributed as dist
except Exception:  # pragma: no cover
    torch = None
    dist = None


class DeepMiner:
    def __init__(self, tx_ptr, items, n_items: int, device: int = 0, rank: int = 0,
                 world: int = 1, comm_backend: Optional[str] = None, **opts):
        self.N = native.require_gpu()
        self.rank, self.world, self.device = rank, world, device
        self.opts = dict(opts)
        self.comm = None
        if world > 1:
            backend = comm_backend or os.environ.get("KMLS_COMM") or (
                "rccl" if dist is not None and dist.is_initialized() and
                dist.get_backend() == "nccl" else "host")
            make_uid = self.N.host_comm_unique_id if backend == "host" else self.N.comm_unique_id
            uid = [make_uid() if rank == 0 else b"\0" * 128]
            dist.broadcast_object_list(uid, src=0)
            self.comm = self.N.Comm(rank, world, uid[0], device, backend)
            self.comm_backend = backend
        else:
            self.comm_backend = None
        self.g = self.N.GpuMiner(device)
        self.g.load_csr(tx_ptr, items, n_items)

    def mine(self, min_support: float, max_len: int = 0) -> Dict:
        """Whole-problem result on every rank (per_level, n_itemsets, digest, ...)."""
        return self.g.mine_deep(min_support, max_len, self.rank, self.world, self.comm,
                                **self.opts)

    def synchronize(self) -> None:
        self.g.synchronize()
