"""Headline step with and without the streamed trie download (PCIe cost of the output)."""
import json
import time

from kubernetes_machine_learning_server_amd.data.synthetic import generate
from kubernetes_machine_learning_server_amd.ops import native

N = native.require_gpu()
tx = generate("ds1", seed=0)
g = N.GpuMiner(0, 0, 0)
g.load_csr(tx.tx_ptr, tx.items, tx.n_items)
for dl in (True, False, True, False):
    for _ in range(5):
        g.mine(0.05, 0, False, dl, True, False, False)
    g.synchronize()
    t0 = time.perf_counter()
    for _ in range(30):
        r = g.mine(0.05, 0, False, dl, True, False, False)
    g.synchronize()
    ms = (time.perf_counter() - t0) * 1000 / 30
    print(json.dumps({"download": dl, "ms_per_step": round(ms, 4), "n": r["stats"]["n_itemsets"],
                      "phases": r["stats"].get("phases_ms")}), flush=True)
