"""One-shot (job) cost of the GPU miner: context + miner construction, CSR upload, first and
second mining call on the headline dataset."""
import json
import time

t0 = time.perf_counter()
from kubernetes_machine_learning_server_amd.data.synthetic import generate  # noqa: E402
from kubernetes_machine_learning_server_amd.ops import native  # noqa: E402

tx = generate("ds1", seed=0)
t1 = time.perf_counter()
N = native.require_gpu()
t2 = time.perf_counter()
g = N.GpuMiner(0)
t3 = time.perf_counter()
g.load_csr(tx.tx_ptr, tx.items, tx.n_items)
t4 = time.perf_counter()
r1 = g.mine(0.05)
t5 = time.perf_counter()
r2 = g.mine(0.05)
t6 = time.perf_counter()
ms = lambda a, b: round((b - a) * 1e3, 2)
print(json.dumps({"import+generate_ms": ms(t0, t1), "require_gpu_ms": ms(t1, t2),
                  "miner_ctor_ms": ms(t2, t3), "arena_gb": round(g.arena_capacity / 2**30, 1),
                  "load_csr_ms": ms(t3, t4), "first_mine_ms": ms(t4, t5),
                  "second_mine_ms": ms(t5, t6), "first_path": r1["stats"]["levels_path"],
                  "first_phases": r1["stats"]["phases_ms"]}), flush=True)
