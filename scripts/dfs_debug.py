"""Diagnostic for the persistent DFS kernel: small cases, tight timeouts, ctl dump per launch."""
import os
import sys
import time

os.environ.setdefault("KMLS_DFS_DEBUG", "1")
os.environ.setdefault("KMLS_DFS_TIMEOUT_MS", "3000")
import numpy as np  # noqa: E402
from kubernetes_machine_learning_server_amd.data.synthetic import generate  # noqa: E402
from kubernetes_machine_learning_server_amd.ops import native  # noqa: E402

N = native.require_gpu()
for shape, ms in [("tiny", 0.1), ("tiny", 0.05), ("ds2_weak", 0.05), ("ds2", 0.06), ("ds2", 0.05)]:
    tx = generate(shape, seed=21)
    c = N.mine_cpu(tx.tx_ptr, tx.items, tx.n_items, ms)
    g = N.GpuMiner(0, 2 << 30, 0)
    g.load_csr(tx.tx_ptr, tx.items, tx.n_items)
    lw = g.mine(ms, persistent=False)
    print(f"{shape}@{ms}: cpu={c['stats']['n_itemsets']} levelwise={lw['stats']['n_itemsets']}", flush=True)
    t = time.perf_counter()
    try:
        p = g.mine(ms, persistent=True)
        print(f"   persistent={p['stats']['n_itemsets']} in {time.perf_counter()-t:.3f}s", flush=True)
    except Exception as e:
        print(f"   persistent FAILED after {time.perf_counter()-t:.3f}s: {e}", flush=True)
        sys.exit(3)
