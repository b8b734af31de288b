#!/usr/bin/env python3
"""Kernel time summary (markdown) from a rocprofv3 rocpd database (run_results.db).

  python scripts/rocpd_summary.py gpurun_out/ktrace_deep/run_results.db > profiles/x.md
"""
import sqlite3
import sys


def main() -> int:
    c = sqlite3.connect(sys.argv[1])
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    rows = c.execute(f"select {name}, count(*), sum(end - start), min(end - start), "
                     f"max(end - start) from kernels group by {name} "
                     f"order by sum(end - start) desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    print("| kernel | calls | total ms | % | min us | max us |")
    print("|---|---|---|---|---|---|")
    for n, k, s, lo, hi in rows:
        short = n if len(n) < 70 else n[:67] + "..."
        print(f"| `{short}` | {k} | {s / 1e6:.3f} | {100 * s / tot:.1f} | {lo / 1e3:.1f} | "
              f"{hi / 1e3:.1f} |")
    return 0


if __name__ == "__main__":
    sys.exit(main())
