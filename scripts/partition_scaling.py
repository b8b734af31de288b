"""Per-rank cost of the replicated multi-GPU mode on one GPU: time GpuMiner.mine_partition for
every rank of world sizes 1, 2, 4, 8 on the headline dataset, with each call waited for ("sync")
and with launch-ahead steady-state calls ("pipelined", bench.py's loop).  The slowest rank bounds a real
N-GPU step (plus one all-reduce), so this predicts the driver's scaling curve."""
import json
import time

from kubernetes_machine_learning_server_amd.data.synthetic import generate
from kubernetes_machine_learning_server_amd.ops import native

N = native.require_gpu()
tx = generate("ds1", seed=0)
g = N.GpuMiner(0, 0, 0)
g.load_csr(tx.tx_ptr, tx.items, tx.n_items)
out = {}
for world in (1, 2, 4, 8):
    res = {}
    for mode in ("sync", "pipelined"):
        per_rank = []
        total = 0
        for rank in range(world):
            pre = mode == "pipelined"
            for i in range(4):
                g.mine_partition(0.05, download=True, rank=rank, world=world, prefetch=pre and i < 3)
            t0 = time.perf_counter()
            for i in range(20):
                r = g.mine_partition(0.05, download=True, rank=rank, world=world,
                                     prefetch=pre and i < 19)
            per_rank.append((time.perf_counter() - t0) * 50.0)
            total += r["stats"]["n_itemsets"]
        res[mode] = {"max_rank_ms": round(max(per_rank), 4), "min_rank_ms": round(min(per_rank), 4),
                     "itemsets": total,
                     "predicted_itemsets_per_s": round(total / (max(per_rank) / 1000.0), 1)}
    out[world] = res
    print(json.dumps({"world": world, **res}), flush=True)
