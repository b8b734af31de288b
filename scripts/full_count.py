#!/usr/bin/env python3
"""Exact COMPLETE count of BASELINE config 2 (ds1 @ 0.01, every itemset of every size), too large
for one bench step: the level-3 tasks are dealt to `world` virtual ranks exactly as a real split
deals them (cost-ordered snake deal) and the ranks are mined one call at a time on one GPU.  Each
rank's partial (per-size counts, digest terms, candidates, seconds) is appended to a JSONL file,
so the count can be spread over several GPU sessions (ranks already in the file are skipped);
when every rank is present the partials are combined (parallel.deep.combine_partials: the same
combine the collectives compute) into the whole-problem result.

  python scripts/full_count.py --world 64 --ranks 0-15 --out profiles/config2_full_partials.jsonl
  python scripts/full_count.py --world 64 --combine --out profiles/config2_full_partials.jsonl
"""
import argparse
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def load(path):
    got = {}
    if os.path.exists(path):
        for line in open(path):
            if line.strip():
                d = json.loads(line)
                got[(d["world"], d["rank"], d["min_support"])] = d
    return got


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--support", type=float, default=0.01)
    ap.add_argument("--world", type=int, default=64)
    ap.add_argument("--ranks", default="", help="a-b (inclusive) of the virtual ranks to mine")
    ap.add_argument("--out", required=True)
    ap.add_argument("--budget", type=float, default=0.0, help="stop starting ranks after N s")
    ap.add_argument("--combine", action="store_true")
    a = ap.parse_args()
    got = load(a.out)
    if a.combine:
        from kubernetes_machine_learning_server_amd.parallel.deep import combine_partials
        parts = [got.get((a.world, r, a.support)) for r in range(a.world)]
        missing = [r for r, p in enumerate(parts) if p is None]
        if missing:
            print(json.dumps({"complete": False, "missing_ranks": missing}))
            return 1
        d = combine_partials(parts)
        secs = [p["s"] for p in parts]
        print(json.dumps({"config": "ds1-shape @ min_support %g, every size" % a.support,
                          "complete": True, "world_virtual": a.world,
                          "n_itemsets": d["n_itemsets"], "max_depth": d["max_depth"],
                          "per_level": d["per_level"], "digest": d["digest"],
                          "candidates": d["candidates"], "one_gpu_s": round(sum(secs), 3),
                          "itemsets_per_s": round(d["n_itemsets"] / sum(secs), 1),
                          "slowest_rank_s": round(max(secs), 3)}))
        return 0
    from kubernetes_machine_learning_server_amd.data.synthetic import generate
    from kubernetes_machine_learning_server_amd.ops import native
    N = native.require_gpu()
    tx = generate("ds1", seed=0)
    g = N.GpuMiner(0)
    g.load_csr(tx.tx_ptr, tx.items, tx.n_items)
    lo, hi = (int(x) for x in a.ranks.split("-"))
    stop = threading.Event()
    t0 = time.time()
    cur = [None]

    def beat():
        while not stop.wait(20):
            print(f"[full_count] {time.time() - t0:.0f} s, rank {cur[0]}", file=sys.stderr,
                  flush=True)
    threading.Thread(target=beat, daemon=True).start()
    try:
        for r in range(lo, hi + 1):
            if (a.world, r, a.support) in got:
                continue
            if a.budget and time.time() - t0 > a.budget:
                break
            cur[0] = r
            t = time.perf_counter()
            d = g.mine_deep(a.support, 0, r, a.world, None, deal_key=0)  # (profiles/config2_full)
            s = time.perf_counter() - t
            rec = {"world": a.world, "rank": r, "min_support": a.support, "s": round(s, 4),
                   "n_itemsets": int(d["n_itemsets"]),
                   "per_level": [int(v) for v in d["per_level"]], "digest": d["digest"],
                   "candidates": int(d["candidates"])}
            with open(a.out, "a") as f:
                f.write(json.dumps(rec) + "\n")
            print(json.dumps(rec), flush=True)
    finally:
        stop.set()
    return 0


if __name__ == "__main__":
    sys.exit(main())
