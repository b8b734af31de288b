"""Config 5 (100M x 1M @2e-4): the deployed rule map through bench_large.run_rule_map (the
bench.py config5 section), one JSON line.  GPU box only.

    python scripts/c5_probe.py [--steps 3] [--hooks pair_rows=0]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, ".")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--hooks", default="")
    a = ap.parse_args()
    if a.hooks:
        os.environ["KMLS_TEST_HOOKS"] = a.hooks
    from kubernetes_machine_learning_server_amd.bench.bench_large import run_rule_map
    print(json.dumps(run_rule_map("100Mx1M", min_support=2e-4, steps=a.steps, warmup=1)), flush=True)


if __name__ == "__main__":
    main()
