"""Per-kernel time summary of a rocprofv3 rocpd database (the .db written by --kernel-trace):
name, calls, total ms, mean/min/max us, sorted by total.  Host-side helper.

    python scripts/rocpd_stats.py gpurun_out/x/serve_results.db [--top 30] [--md]
"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--md", action="store_true")
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "name" if "name" in cols else "kernel_name"
    rows = c.execute(f"select {name}, count(*), sum(end-start), min(end-start), max(end-start) "
                     f"from kernels group by {name} order by sum(end-start) desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    if a.md:
        print("| kernel | calls | total ms | % | mean us | min us | max us |")
        print("|---|---|---|---|---|---|---|")
    for n, k, s, mn, mx in rows[:a.top]:
        if a.match and a.match not in n:
            continue
        short = n if len(n) < 90 else n[:87] + "..."
        if a.md:
            print(f"| `{short}` | {k} | {s / 1e6:.3f} | {100 * s / tot:.1f} | {s / k / 1e3:.1f} | "
                  f"{mn / 1e3:.1f} | {mx / 1e3:.1f} |")
        else:
            print(f"{s / 1e6:10.3f} ms {k:7d} x {s / k / 1e3:9.1f} us (min {mn / 1e3:.1f}, max "
                  f"{mx / 1e3:.1f})  {short}")


if __name__ == "__main__":
    main()
