"""A/B sweep of the deep miner's stealing knobs (env-read per call) at a simulated rank split:
one JSON line per configuration with every rank's time and the slowest.  GPU box only.

    python scripts/deep_sweep_env.py --world 8 --configs "BUDGET=8;BUDGET=16;STEAL_IDLE=1,SPLIT_MIN=2"
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

KEYS = {}  # env-read knobs (none at the moment); the rest go to mine_deep


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--support", type=float, default=0.02)
    ap.add_argument("--reps", type=int, default=1)
    ap.add_argument("--budget", type=int, default=0)
    ap.add_argument("--configs", required=True)
    a = ap.parse_args()
    from kubernetes_machine_learning_server_amd.data.synthetic import generate
    from kubernetes_machine_learning_server_amd.ops import native
    N = native.require_gpu()
    tx = generate("ds1", seed=0)
    g = N.GpuMiner(0)
    g.load_csr(tx.tx_ptr, tx.items, tx.n_items)
    kw = {"budget": a.budget} if a.budget else {}
    g.mine_deep(a.support, 0, rank=0, world=a.world, **kw)  # cold call
    for cfg in a.configs.split(";"):
        for v in KEYS.values():
            os.environ.pop(v, None)
        for kv in filter(None, cfg.split(",")):
            k, v = kv.split("=")
            if k == "BUDGET":
                kw["budget"] = int(v)
                continue
            if k in ("STEAL_IDLE", "PRESPLIT_COST", "BLOCKS_PER_CU", "SPLIT_MIN"):
                kw[k.lower()] = int(v)
                continue
            os.environ[KEYS[k]] = v
        best = None
        for _ in range(a.reps):
            ranks, n = [], 0
            for r in range(a.world):
                d = g.mine_deep(a.support, 0, rank=r, world=a.world, **kw)
                ranks.append(round(d["phases_ms"]["total"], 3))
                n += d["n_itemsets"]
            if best is None or max(ranks) < max(best):
                best = ranks
        print(json.dumps({"cfg": cfg, "world": a.world, "slowest_ms": max(best), "ranks_ms": best,
                          "n": n}), flush=True)
        kw = {"budget": a.budget} if a.budget else {}


if __name__ == "__main__":
    main()
