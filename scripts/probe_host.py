"""Host-side overhead of one headline mining call: Python wall per call vs the C++ call's own
wall time (stats.seconds), GPU phases (hipEvent-timed) and the host_* phases."""
import json
import time

import numpy as np

from kubernetes_machine_learning_server_amd.data.synthetic import generate
from kubernetes_machine_learning_server_amd.ops import native

N = native.require_gpu()
tx = generate("ds1", seed=0)
g = N.GpuMiner(0, 0, 0)
g.load_csr(tx.tx_ptr, tx.items, tx.n_items)
for _ in range(5):
    g.mine(0.05, 0, False, True, True, False, False)
wall, cpp, ph = [], [], {}
for _ in range(50):
    t0 = time.perf_counter()
    r = g.mine(0.05, 0, False, True, True, False, False)
    wall.append(time.perf_counter() - t0)
    st = r["stats"]
    cpp.append(st["seconds"])
    for k, v in st["phases_ms"].items():
        ph.setdefault(k, []).append(v * 1000.0)
f = lambda v: round(float(np.median(v)) * 1e6, 1)
out = {"python_wall_us": f(wall), "cpp_call_us": f(cpp)}
out.update({k + "_us": round(float(np.median(v)), 1) for k, v in ph.items()})
print(json.dumps(out), flush=True)
