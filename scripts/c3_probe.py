"""Config 3 (10M x 1M @2e-4, tx-DP at world 1) through bench_mine.run_config3: one JSON line with
the step time, phases, horizontal-level stats and the digest.  GPU box only.

    python scripts/c3_probe.py [--steps 5] [--hooks cooc=2] [--min-support 7e-5]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, ".")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--hooks", default="")
    ap.add_argument("--shape", default="10Mx1M", help="100Mx1M: config 5's data, every size")
    ap.add_argument("--min-support", type=float, default=0.0,
                    help="0 = the config's 2e-4; 7e-5 gives ~59.7k frequent items")
    a = ap.parse_args()
    if a.hooks:
        os.environ["KMLS_TEST_HOOKS"] = a.hooks
    from kubernetes_machine_learning_server_amd.bench import bench_mine as bm
    from kubernetes_machine_learning_server_amd.ops import native
    N = native.require_gpu()
    kw = {"min_support": a.min_support} if a.min_support else {}
    kw["shape_name"] = a.shape
    out = bm.run_config3(N, 1, 0, 0, steps=a.steps, warmup=1, **kw)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
