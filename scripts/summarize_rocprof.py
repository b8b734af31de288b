#!/usr/bin/env python3
"""Summarise a rocprofv3 --stats kernel_stats.csv into a short markdown table."""
import csv
import re
import sys


def short(name: str) -> str:
    if "rocprim" in name:
        return "rocprim::" + ("init_lookback_scan_state" if "init_lookback" in name else "device_scan")
    m = re.search(r"(k_[a-z0-9_]+(<\d+>)?)", name)
    return m.group(1) if m else name.split("(")[0][-50:]


def main(path, steps=None):
    rows = list(csv.DictReader(open(path)))
    agg = {}
    for r in rows:
        k = short(r["Name"])
        a = agg.setdefault(k, [0, 0.0])
        a[0] += int(r["Calls"])
        a[1] += float(r["TotalDurationNs"])
    tot = sum(v[1] for v in agg.values())
    print(f"| kernel | calls | total ms | avg us | % |")
    print(f"|---|---|---|---|---|")
    for k, (c, ns) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"| {k} | {c} | {ns/1e6:.3f} | {ns/c/1e3:.2f} | {100*ns/tot:.1f} |")
    print(f"\ntotal GPU kernel+copy time: {tot/1e6:.3f} ms"
          + (f" over {steps} steps = {tot/1e6/steps:.3f} ms/step" if steps else ""))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else None)
