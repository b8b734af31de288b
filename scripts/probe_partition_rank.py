"""Steady-state cost of ONE rank of the replicated multi-GPU mode on one GPU (the driver's
N-GPU bench runs each rank on its own GPU): repeated mine_partition(rank, world) calls, so the
per-level launch hints are the rank's own.  Usage: probe_partition_rank.py <world> [rank|max]"""
import json
import sys
import time

from kubernetes_machine_learning_server_amd.data.synthetic import generate
from kubernetes_machine_learning_server_amd.ops import native

world = int(sys.argv[1]) if len(sys.argv) > 1 else 8
which = sys.argv[2] if len(sys.argv) > 2 else "max"
N = native.require_gpu()
tx = generate("ds1", seed=0)
out = []
ranks = range(world) if which == "max" else [int(which)]
for rank in ranks:
    g = N.GpuMiner(0, 0, 0)  # one miner per rank, as on a real node
    g.load_csr(tx.tx_ptr, tx.items, tx.n_items)
    for _ in range(5):
        g.mine_partition(0.05, 0, True, rank, world)
    t0 = time.perf_counter()
    for _ in range(30):
        r = g.mine_partition(0.05, 0, True, rank, world)
    ms = (time.perf_counter() - t0) * 1000 / 30
    out.append({"rank": rank, "ms": round(ms, 4), "itemsets": r["stats"]["n_itemsets"],
                "depth": r["stats"]["max_depth"]})
    del g
print(json.dumps({"world": world, "ranks": out,
                  "max_ms": max(o["ms"] for o in out),
                  "itemsets": sum(o["itemsets"] for o in out)}), flush=True)
