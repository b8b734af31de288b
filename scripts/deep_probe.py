#!/usr/bin/env python3
"""Probe of the count-only deep miner on ds1: parity at 0.03 against the CPU count, then timed
full mining at lower supports (the BASELINE config-2 family), one JSON line per run.

  python scripts/deep_probe.py --supports 0.02 --reps 3 [--budget 4096 --budget0 4096]
  python scripts/deep_probe.py --sweep 4096:4096:4:3,1024:1024:4:3 --supports 0.02
      (budget0:budget:split_min:blocks_per_cu per config, min of --reps per config)
  python scripts/deep_probe.py --world 8 --supports 0.02   (every rank's share, one GPU)

A heartbeat line goes to stderr every 30 s while a call runs (long runs at 0.015 and below).
"""
import argparse
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# CPU references (mine_cpu_count on the build host, 6 threads; profiles/r3_config2_cpu_ref.md)
CPU_REF = {
    0.02: ("1d15b1d026fe928d14a65f5b88be8656", 1414082373),
}


class Heartbeat:
    def __init__(self, what: str, every: float = 30.0):
        self.what, self.every, self.stop = what, every, threading.Event()
        self.t = threading.Thread(target=self._run, daemon=True)

    def _run(self):
        t0 = time.time()
        while not self.stop.wait(self.every):
            print(f"[deep_probe] {self.what}: {time.time() - t0:.0f} s", file=sys.stderr,
                  flush=True)

    def __enter__(self):
        self.t.start()
        return self

    def __exit__(self, *a):
        self.stop.set()


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--supports", default="0.02")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--budget", type=int, default=0)
    ap.add_argument("--budget0", type=int, default=0)
    ap.add_argument("--split-min", type=int, default=0)
    ap.add_argument("--blocks-per-cu", type=int, default=0)
    ap.add_argument("--max-len", type=int, default=0)
    ap.add_argument("--sweep", default="",
                    help="b0:b:split:bpc[:steal[:steal_idle]],... configurations")
    ap.add_argument("--rounds", action="store_true", help="spill rounds instead of stealing")
    ap.add_argument("--world", type=int, default=1, help="simulate a rank split on one GPU")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--assign", type=int, default=1,
                    help="level-3 task assignment: 1 = cost-ordered snake deal, 0 = t mod world")
    ap.add_argument("--trace", action="store_true", help="per-wave / per-task timing summary")
    ap.add_argument("--presplit-cost", type=int, default=16, help="0 = no pre-split launch")
    ap.add_argument("--presplit-budget", type=int, default=1)
    ap.add_argument("--emit", action="store_true",
                    help="materialise every itemset (the bench's emit block; digest = arena's)")
    a = ap.parse_args()
    from kubernetes_machine_learning_server_amd.data.synthetic import generate
    from kubernetes_machine_learning_server_amd.ops import native
    N = native.require_gpu()
    tx = generate("ds1", seed=0)
    g = N.GpuMiner(0)
    g.load_csr(tx.tx_ptr, tx.items, tx.n_items)

    def opts(b0, b, sm, bpc, steal=1, idle=1):
        kw = {"steal": bool(steal), "steal_idle": idle}
        for k, v in (("budget0", b0), ("budget", b), ("split_min", sm), ("blocks_per_cu", bpc)):
            if v:
                kw[k] = v
        return kw

    kw = opts(a.budget0, a.budget, a.split_min, a.blocks_per_cu, 0 if a.rounds else 1)
    kw["assign"] = a.assign
    kw["trace"] = a.trace
    kw["presplit_cost"] = a.presplit_cost
    kw["presplit_budget"] = a.presplit_budget
    kw["emit"] = a.emit
    if not a.no_parity:
        t = time.perf_counter()
        d = g.mine_deep(0.03, **kw)
        dt = time.perf_counter() - t
        c = N.mine_cpu_count(tx.tx_ptr, tx.items, tx.n_items, 0.03)
        print(json.dumps({"probe": "parity", "min_support": 0.03, "n": d["n_itemsets"],
                          "ok": d["digest"] == c["digest"] and d["n_itemsets"] == c["n_itemsets"],
                          "s": round(dt, 4), "phases_ms": d["phases_ms"],
                          "rounds": len(d["round_tasks"])}), flush=True)
    if a.sweep:
        for cfg in a.sweep.split(","):
            k = opts(*(int(x) for x in cfg.split(":")))
            for ms in [float(x) for x in a.supports.split(",")]:
                best, d = None, None
                for _ in range(a.reps):
                    t = time.perf_counter()
                    d = g.mine_deep(ms, a.max_len, **k)
                    dt = time.perf_counter() - t
                    best = dt if best is None else min(best, dt)
                ref = CPU_REF.get(ms)
                print(json.dumps({"probe": "sweep", "cfg": cfg, "min_support": ms,
                                  "best_s": round(best, 4), "n": d["n_itemsets"],
                                  "ok": (d["digest"] == ref[0]) if ref and not a.max_len else None,
                                  "chunks": d["chunks"], "n_rounds": len(d["round_tasks"]),
                                  "spilled": d["spilled_tasks"], "handoffs": d["handoffs"],
                                  "round_ms": [round(x, 1) for x in d["round_ms"][:12]]}),
                      flush=True)
        return 0
    for ms in [float(x) for x in a.supports.split(",")]:
        # one untimed call first: the first call allocates the miner's buffers (the cold call is
        # what is dropped, not a rank)
        g.mine_deep(ms, a.max_len, rank=0, world=a.world, **kw)
        for rep in range(a.reps):
            comb = {"sum": 0, "xor": 0, "n": 0, "slowest_ms": 0.0, "ranks_ms": []}
            for r in range(a.world):
                t = time.perf_counter()
                with Heartbeat(f"min_support {ms} rank {r}"):
                    d = g.mine_deep(ms, a.max_len, rank=r, world=a.world, **kw)
                dt = time.perf_counter() - t
                ref = CPU_REF.get(ms)
                out = {"probe": "deep", "min_support": ms, "rep": rep, "rank": r,
                       "world": a.world, "s": round(dt, 4), "n": d["n_itemsets"],
                       "itemsets_per_s": round(d["n_itemsets"] / dt, 1),
                       "per_level": d["per_level"][1:], "digest": d["digest"],
                       "candidates": d["candidates"], "chunks": d["chunks"],
                       "level2_tasks": d["level2_tasks"], "phases_ms": d["phases_ms"],
                       "round_tasks": d["round_tasks"][:12],
                       "round_ms": [round(x, 2) for x in d["round_ms"][:12]],
                       "n_rounds": len(d["round_tasks"]), "spilled": d["spilled_tasks"],
                       "handoffs": d["handoffs"], "presplit": d.get("presplit")}
                if ref and a.world == 1 and not a.max_len:
                    out["verified_vs_cpu"] = d["digest"] == ref[0] and d["n_itemsets"] == ref[1]
                if a.trace:
                    out["trace"] = trace_summary(d)
                print(json.dumps(out), flush=True)
                comb["sum"] = (comb["sum"] + int(d["digest"][:16], 16)) % (1 << 64)
                comb["xor"] ^= int(d["digest"][16:], 16)
                comb["n"] += d["n_itemsets"]
                comb["slowest_ms"] = max(comb["slowest_ms"], d["phases_ms"]["total"])
                comb["ranks_ms"].append(round(d["phases_ms"]["total"], 3))
            if a.world > 1:
                dg = f"{comb['sum']:016x}{comb['xor']:016x}"
                ref = CPU_REF.get(ms)
                print(json.dumps({"probe": "split", "min_support": ms, "rep": rep,
                                  "world": a.world, "assign": a.assign,
                                  "presplit_cost": a.presplit_cost, "n": comb["n"],
                                  "digest": dg,
                                  "verified_vs_cpu": (dg == ref[0] and comb["n"] == ref[1])
                                  if ref and not a.max_len else None,
                                  "slowest_rank_ms": round(comb["slowest_ms"], 3),
                                  "ranks_ms": comb["ranks_ms"]}),
                      flush=True)
    return 0


def trace_summary(d):
    """Tail analysis of one stealing launch from the per-wave / per-task timing."""
    import numpy as np
    tr = np.asarray(d["trace"], np.int64)
    if tr.size == 0:
        return None
    tick_ms = 1.0 / float(d["clock_khz"])
    t0 = tr[:, 0].min()
    span = (tr[:, 3].max() - t0) * tick_ms
    first = (tr[:, 1] - t0) * tick_ms
    last = (tr[:, 2] - t0) * tick_ms
    busy = tr[:, 4] * tick_ms
    tasks = tr[:, 5] >> 32
    inbox = tr[:, 5] & 0xffffffff
    pct = lambda x: [round(float(np.percentile(x, q)), 3) for q in (0, 10, 50, 90, 100)]
    bw = float(d.get("trace_bucket", 0) or 0)
    curve = None
    if bw and tr.shape[1] > 6:
        # fraction of the waves busy in each time bucket (the launch's activity profile)
        nb = int(np.ceil(span / (bw * tick_ms)))
        curve = [round(float(x), 3) for x in (tr[:, 6:6 + nb].sum(0) / (bw * len(tr)))]
    drain = (float(d["t_drain"]) - t0) * tick_ms if d.get("t_drain") else None
    out = {"span_ms": round(span, 3), "busy_frac": round(float(busy.sum() / (len(tr) * span)), 3),
           "bucket_ms": round(bw * tick_ms, 3) if bw else None, "busy_curve": curve,
           "queue_drained_ms": round(drain, 3) if drain is not None else None,
           "first_task_start_ms_pctl": pct(first), "last_task_end_ms_pctl": pct(last),
           "tasks_per_wave_pctl": pct(tasks), "inbox_per_wave_pctl": pct(inbox)}
    tk = np.asarray(d.get("task_ticks", []), np.int64) * tick_ms
    cost = np.asarray(d.get("task_cost", []), np.int64)
    if tk.size and cost.size == tk.size:
        bins = {}
        for lo, hi in ((0, 1), (1, 4), (4, 16), (16, 64), (64, 256), (256, 1 << 30)):
            m = (cost >= lo) & (cost < hi)
            if m.any():
                bins[f"{lo}-{hi}"] = [int(m.sum()), round(float(tk[m].mean()), 4),
                                      round(float(tk[m].max()), 3)]
        out["task_ms_by_cost"] = bins  # [tasks, mean ms, max ms] (own work, hand-offs excluded)
        top = np.argsort(-tk)[:8]
        out["top_tasks"] = [[int(q), int(cost[q]), round(float(tk[q]), 3)] for q in top]
    return out


if __name__ == "__main__":
    sys.exit(main())
