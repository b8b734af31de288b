#!/usr/bin/env python3
"""Per-step kernel timeline (and optional HIP API summary) from a rocprofv3 rocpd SQLite DB.

Usage: rocpd_timeline.py <run_results.db> [--marker k_item_support] [--step -2] [--api]

Steps are delimited by the first kernel of a mining call (``--marker``).  Prints one row per
kernel of the chosen step (start/end relative to the step start, duration, queue, grid,
register and LDS use), the GPU-idle time inside the step, and — with ``--api`` — the HIP API
calls issued between the two step markers, aggregated by name (count, total us)."""
import argparse
import re
import sqlite3


def short(n: str) -> str:
    m = re.search(r"(k_[a-z0-9_]+(<\d+>)?)", n)
    return m.group(1) if m else n.split("(")[0][:40]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--marker", default="k_item_support")
    ap.add_argument("--step", type=int, default=-2, help="index of the step (python-style)")
    ap.add_argument("--api", action="store_true")
    a = ap.parse_args()
    db = sqlite3.connect(a.db)
    cur = db.cursor()
    rows = list(cur.execute("select name,start,end,queue_id,grid_x,vgpr_count,sgpr_count,lds_size "
                            "from kernels order by start"))
    idx = [i for i, r in enumerate(rows) if a.marker in r[0]]
    if len(idx) < 2:
        raise SystemExit("fewer than two step markers")
    starts = idx + [len(rows)]
    k = a.step if a.step >= 0 else len(idx) + a.step
    s, e = starts[k], starts[k + 1]
    t0 = rows[s][1]
    t_end = rows[e][1] if e < len(rows) else max(r[2] for r in rows[s:e])
    print("| kernel | queue | start us | end us | dur us | grid | vgpr | sgpr | lds |")
    print("|---|---|---|---|---|---|---|---|---|")
    busy = []
    for r in rows[s:e]:
        print(f"| {short(r[0])} | {r[3]} | {(r[1]-t0)/1e3:.1f} | {(r[2]-t0)/1e3:.1f} | "
              f"{(r[2]-r[1])/1e3:.1f} | {r[4]} | {r[5]} | {r[6]} | {r[7]} |")
        busy.append((r[1], r[2]))
    busy.sort()
    covered, cur_s, cur_e = 0, None, None
    for bs, be in busy:
        if cur_e is None or bs > cur_e:
            if cur_e is not None:
                covered += cur_e - cur_s
            cur_s, cur_e = bs, be
        else:
            cur_e = max(cur_e, be)
    if cur_e is not None:
        covered += cur_e - cur_s
    span = t_end - t0
    print(f"\nstep span {span/1e3:.1f} us, GPU busy {covered/1e3:.1f} us, idle {(span-covered)/1e3:.1f} us")
    if a.api:
        try:
            api = list(cur.execute("select name,start,end from regions where start>=? and start<? "
                                   "order by start", (t0 - 2_000_000, t_end)))
        except sqlite3.OperationalError as ex:
            raise SystemExit(f"no API regions in this DB ({ex})")
        agg = {}
        for n, bs, be in api:
            v = agg.setdefault(n, [0, 0])
            v[0] += 1
            v[1] += be - bs
        print("\n| HIP API | calls | total us |\n|---|---|---|")
        for n, (c, ns) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
            print(f"| {n} | {c} | {ns/1e3:.1f} |")


if __name__ == "__main__":
    main()
