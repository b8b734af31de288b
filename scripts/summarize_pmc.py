#!/usr/bin/env python3
"""Aggregate a rocprofv3 --pmc counter_collection.csv per kernel (sum over dispatches) into a
markdown table; derived: MFMA busy % of CU busy cycles, i8 MFMA ops/s over kernel time."""
import csv
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    m = re.search(r"(k_[a-z0-9_]+(<\d+>)?)", name)
    return m.group(1) if m else name.split("(")[0][-40:]


def main(path: str) -> None:
    rows = list(csv.DictReader(open(path)))
    if not rows:
        print("no rows")
        return
    kcol = next(c for c in rows[0] if c.lower() in ("kernel_name", "kernel-name", "name"))
    ccol = next(c for c in rows[0] if c.lower() in ("counter_name", "counter-name"))
    vcol = next(c for c in rows[0] if c.lower() in ("counter_value", "counter-value", "value"))
    agg = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for r in rows:
        k = short(r[kcol])
        agg[k][r[ccol]] += float(r[vcol])
        disp[k].add(r.get("Dispatch_Id") or r.get("dispatch_id") or len(disp[k]))
    counters = sorted({c for v in agg.values() for c in v})
    print("| kernel | dispatches | " + " | ".join(counters) + " |")
    print("|---|---|" + "---|" * len(counters))
    for k, v in sorted(agg.items(), key=lambda kv: -max(kv[1].values())):
        print(f"| {k} | {len(disp[k])} | " + " | ".join(f"{v.get(c, 0):.4g}" for c in counters) + " |")
    for k, v in agg.items():
        if v.get("SQ_VALU_MFMA_BUSY_CYCLES") and v.get("SQ_BUSY_CU_CYCLES"):
            print(f"\n{k}: MFMA busy / CU busy = "
                  f"{100.0 * v['SQ_VALU_MFMA_BUSY_CYCLES'] / v['SQ_BUSY_CU_CYCLES']:.1f} %")


if __name__ == "__main__":
    main(sys.argv[1])
