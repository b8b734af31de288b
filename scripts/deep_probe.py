#!/usr/bin/env python3
"""Probe of the count-only deep miner on ds1: parity at 0.03 against the CPU count, then timed
full mining at lower supports (the BASELINE config-2 family), one JSON line per run.

  python scripts/deep_probe.py --supports 0.02 --reps 3 [--budget 4096 --budget0 4096]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# CPU references (mine_cpu_count on the build host, 6 threads; profiles/r3_config2_cpu_ref.md)
CPU_REF = {
    0.02: ("5645ebcc74e7a31e9f474dfbb0c9e0bb", 1414082373),
}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--supports", default="0.02")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--budget", type=int, default=4096)
    ap.add_argument("--budget0", type=int, default=4096)
    ap.add_argument("--split-min", type=int, default=4)
    ap.add_argument("--blocks-per-cu", type=int, default=0)
    ap.add_argument("--world", type=int, default=1, help="simulate a rank split on one GPU")
    ap.add_argument("--no-parity", action="store_true")
    a = ap.parse_args()
    from kubernetes_machine_learning_server_amd.data.synthetic import generate
    from kubernetes_machine_learning_server_amd.ops import native
    N = native.require_gpu()
    tx = generate("ds1", seed=0)
    g = N.GpuMiner(0)
    g.load_csr(tx.tx_ptr, tx.items, tx.n_items)
    kw = dict(budget0=a.budget0, budget=a.budget, split_min=a.split_min,
              blocks_per_cu=a.blocks_per_cu)
    if not a.no_parity:
        t = time.perf_counter()
        d = g.mine_deep(0.03, **kw)
        dt = time.perf_counter() - t
        c = N.mine_cpu_count(tx.tx_ptr, tx.items, tx.n_items, 0.03)
        print(json.dumps({"probe": "parity", "min_support": 0.03, "n": d["n_itemsets"],
                          "ok": d["digest"] == c["digest"] and d["n_itemsets"] == c["n_itemsets"],
                          "s": round(dt, 4), "phases_ms": d["phases_ms"],
                          "rounds": len(d["round_tasks"])}), flush=True)
    for ms in [float(x) for x in a.supports.split(",")]:
        for rep in range(a.reps):
            for r in range(a.world):
                t = time.perf_counter()
                d = g.mine_deep(ms, rank=r, world=a.world, **kw)
                dt = time.perf_counter() - t
                ref = CPU_REF.get(ms)
                out = {"probe": "deep", "min_support": ms, "rep": rep, "rank": r,
                       "world": a.world, "s": round(dt, 4), "n": d["n_itemsets"],
                       "itemsets_per_s": round(d["n_itemsets"] / dt, 1),
                       "per_level": d["per_level"][1:], "digest": d["digest"],
                       "candidates": d["candidates"], "chunks": d["chunks"],
                       "level2_tasks": d["level2_tasks"], "phases_ms": d["phases_ms"],
                       "round_tasks": d["round_tasks"][:12],
                       "round_ms": [round(x, 2) for x in d["round_ms"][:12]],
                       "n_rounds": len(d["round_tasks"])}
                if ref and a.world == 1:
                    out["verified_vs_cpu"] = d["digest"] == ref[0] and d["n_itemsets"] == ref[1]
                print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
