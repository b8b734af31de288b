"""Per-tile phase timing of one level's count kernel (KMLS_LEVEL_TRACE=<L>, set by the caller):
mines the headline dataset a few times, then summarises the uint64 [tile][8] timestamps the
miner wrote (wall_clock64 ticks, 100 MHz)."""
import json
import os
import sys

import numpy as np

from kubernetes_machine_learning_server_amd.data.synthetic import generate
from kubernetes_machine_learning_server_amd.ops import native

path = os.environ.get("KMLS_LEVEL_TRACE_FILE", "level_trace.bin")
N = native.require_gpu()
tx = generate("ds1", seed=0)
g = N.GpuMiner(0, 0, 0)
g.load_csr(tx.tx_ptr, tx.items, tx.n_items)
for _ in range(4):
    g.mine(0.05, 0, False, True, True, False, False)
tr = np.fromfile(path, dtype=np.uint64).reshape(-1, 8).astype(np.int64)
tr = tr[tr[:, 0] > 0]
t0 = tr[:, 0].min()
us = lambda x: x / 100.0  # 100 MHz ticks → µs
names = ["window", "phase1+scan", "lookback", "phase2", "phase3", "tail", "sync"]
out = {"level": int(os.environ.get("KMLS_LEVEL_TRACE", "0")), "tiles": int(len(tr)),
       "kernel_span_us": us(tr[:, 6].max() - t0),
       "tile_start_us": {"p50": us(np.percentile(tr[:, 0] - t0, 50)),
                         "max": us((tr[:, 0] - t0).max())}}
for k, n in enumerate(names):
    d = us(tr[:, k + 1] - tr[:, k])
    out[n] = {"mean": round(float(d.mean()), 2), "p50": round(float(np.percentile(d, 50)), 2),
              "p90": round(float(np.percentile(d, 90)), 2), "max": round(float(d.max()), 2)}
lb = us(tr[:, 3] - tr[:, 2])
order = np.argsort(np.arange(len(tr)))
out["lookback_by_tile_decile"] = [round(float(x.mean()), 2) for x in np.array_split(lb, 10)]
print(json.dumps(out), flush=True)
