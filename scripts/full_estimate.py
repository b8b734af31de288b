#!/usr/bin/env python3
"""Estimate of the complete config-2 result (ds1 @ 0.01, every size) from exactly mined random
virtual ranks of a cost-dealt split (parallel.deep.estimate_total), and a check of the same
estimator at a size cap where the exact count is known.

  python scripts/full_estimate.py --support 0.01 --world 4096 --samples 16 [--check-len 7]

One JSON line per estimate on stdout; a heartbeat on stderr.
"""
import argparse
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--support", type=float, default=0.01)
    ap.add_argument("--world", type=int, default=4096)
    ap.add_argument("--samples", type=int, default=16)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--budget", type=float, default=120.0, help="seconds of sampling")
    ap.add_argument("--check-len", type=int, default=0,
                    help="also estimate at this size cap and compare with the exact count")
    ap.add_argument("--max-len", type=int, default=0)
    a = ap.parse_args()
    from kubernetes_machine_learning_server_amd.data.synthetic import generate
    from kubernetes_machine_learning_server_amd.ops import native
    from kubernetes_machine_learning_server_amd.parallel.deep import estimate_total
    N = native.require_gpu()
    tx = generate("ds1", seed=0)
    g = N.GpuMiner(0)
    g.load_csr(tx.tx_ptr, tx.items, tx.n_items)
    stop = threading.Event()
    t0 = time.time()

    def beat():
        while not stop.wait(20):
            print(f"[full_estimate] {time.time() - t0:.0f} s", file=sys.stderr, flush=True)
    threading.Thread(target=beat, daemon=True).start()
    try:
        if a.check_len:
            t = time.perf_counter()
            exact = g.mine_deep(a.support, a.check_len)
            ex_s = time.perf_counter() - t
            e = estimate_total(g, a.support, a.world, a.samples, a.seed, a.check_len, a.budget)
            n = int(exact["n_itemsets"])
            e.update(check="estimator vs exact count at a size cap", exact=n,
                     exact_s=round(ex_s, 3), error=e["n_itemsets_estimate"] - n,
                     z=round((e["n_itemsets_estimate"] - n) / e["n_itemsets_se"], 3)
                     if e["n_itemsets_se"] else None)
            print(json.dumps(e), flush=True)
        e = estimate_total(g, a.support, a.world, a.samples, a.seed, a.max_len, a.budget)
        print(json.dumps(e), flush=True)
    finally:
        stop.set()
    return 0


if __name__ == "__main__":
    sys.exit(main())
