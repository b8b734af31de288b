"""Round-trip latency of the persistent serving kernel against the per-batch launch path and the
C++ matcher, single queries and small batches on a ds1 index (GPU box only).

    python scripts/serve_loop_probe.py [--reps 2000]
"""
import argparse
import json
import sys
import time

import numpy as np

sys.path.insert(0, ".")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=2000)
    a = ap.parse_args()
    from kubernetes_machine_learning_server_amd.data.synthetic import generate
    from kubernetes_machine_learning_server_amd.ops import native
    from kubernetes_machine_learning_server_amd.serve.index import build_index_from_trie
    N = native.require_gpu()
    tx = generate("ds1", seed=0)
    r = N.mine_cpu(tx.tx_ptr, tx.items, tx.n_items, 0.03, 2)
    idx = build_index_from_trie(r["parent"], r["item"], r["count"], r["depth"], tx.n_tx, tx.n_items)
    host = idx.native()
    g = N.GpuRuleIndex(0, host)
    keys = np.flatnonzero(idx.is_key).astype(np.int32)
    rng = np.random.default_rng(0)
    for B in (1, 4, 16, 64):
        lens = rng.integers(1, 6, size=B)
        q_ptr = np.zeros(B + 1, np.int64)
        np.cumsum(lens, out=q_ptr[1:])
        seeds = keys[rng.integers(0, len(keys), int(q_ptr[-1]))].astype(np.int32)
        out = {"B": B}
        for name, fn in (("cpp", lambda: host.query_batch(q_ptr, seeds, 10)),
                         ("loop", lambda: g.query_loop(q_ptr, seeds, 10)),
                         ("launch", lambda: g.query_batch(q_ptr, seeds, 10))):
            fn()
            ts = []
            for _ in range(a.reps if name != "launch" else a.reps // 4):
                t0 = time.perf_counter()
                fn()
                ts.append(time.perf_counter() - t0)
            ts = np.asarray(ts) * 1e6
            out[name] = {"p50_us": round(float(np.median(ts)), 2),
                         "p99_us": round(float(np.percentile(ts, 99)), 2)}
        st = N.serve_loop_stats(0)
        out["loop_kernel_mean_us"] = round(st["kernel_mean_us"], 2)
        out["loop_stage_mean_us"] = round(st.get("stage_mean_us", 0.0), 2)
        out["loop_compute_mean_us"] = round(st.get("compute_mean_us", 0.0), 2)
        out["loop_phase_us"] = [round(x, 2) for x in st.get("phase_mean_us", [])]
        out["loop_launches"] = st["launches"]
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
