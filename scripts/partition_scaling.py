"""Per-rank cost of the replicated multi-GPU mode on one GPU: time GpuMiner.mine_partition for
every rank of world sizes 1, 2, 4, 8 on the headline dataset.  The slowest rank bounds a real
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
    per_rank = []
    total = 0
    for rank in range(world):
        for _ in range(3):
            g.mine_partition(0.05, download=True, rank=rank, world=world)
        t0 = time.perf_counter()
        for _ in range(10):
            r = g.mine_partition(0.05, download=True, rank=rank, world=world)
        per_rank.append((time.perf_counter() - t0) * 100.0)
        total += r["stats"]["n_itemsets"]
    out[world] = {"max_rank_ms": round(max(per_rank), 4), "min_rank_ms": round(min(per_rank), 4),
                  "itemsets": total,
                  "predicted_itemsets_per_s": round(total / (max(per_rank) / 1000.0), 1)}
    print(json.dumps({"world": world, **out[world]}), flush=True)
