"""Serving benchmark: p50/p99 latency of POST /api/recommend/ at fixed offered QPS.

BASELINE.json's second metric (config 4: 10k QPS, HBM-resident rule index, 1 MI355X).

* Load: the native open-loop generator (``_native.loadgen``, csrc/host/loadgen.cpp): request i
  is due at t0 + i/QPS on keep-alive connection i % C; latency is measured from that SCHEDULED
  time, so server stalls show up as latency (no coordinated omission).  ``--client python``
  keeps the older aiohttp client processes for comparison.
* Server: ``--front native`` (default; C++ HTTP I/O threads in front of the FastAPI app, GPU
  matching in-process, serve/front.py) or ``--front uvicorn`` (the pure FastAPI stack,
  ``--workers`` processes), over a PVC directory populated by the real job on ds1-shaped data.
* Backends: ``hip`` (every request through the HIP matcher over the HBM index), ``auto`` (HIP
  only for batches past the crossover measured at load), ``cpu`` (C++ matcher), ``python`` (the
  reference's own dict/defaultdict/sorted matcher, rest_api/app/main.py:224-254).
* ``--capacity``: the QPS is raised (x2, then bisected) to the highest rate answered with
  p99 < 5 ms and no errors.
* The bench process never initialises the GPU itself (the PVC is mined by the CPU miner, whose
  artifact is identical): the server is a fresh child process.
* ``--matcher-only``: in-process matcher throughput without HTTP.

  python -m kubernetes_machine_learning_server_amd.bench.bench_serve --backend auto --qps 2000,10000 --capacity
"""
from __future__ import annotations

import argparse
import asyncio
import json
import multiprocessing as mp
import os
import pathlib
import signal
import socket
import subprocess
import sys
import tempfile
import time
from typing import List, Optional

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[2]


def prepare_pvc(root: pathlib.Path, shape: str = "ds1", ms: float = 0.05, miner: str = "cpu"):
    from ..config import JobSettings
    from ..data.synthetic import generate, to_reference_csv
    from ..job import main as job
    ds = root / "datasets"
    ds.mkdir(parents=True, exist_ok=True)
    tx = generate(shape, seed=0)
    to_reference_csv(tx, ds / "2023_spotify_ds1.csv", seed=0)
    base = root / "api-data"
    cfg = JobSettings(min_support=ms, base_dir=base, datasets_dir=ds, pickles_folder=base / "pickles",
                      recommendations_file="recommendations.pickle", best_tracks_file="best_tracks.pickle",
                      data_invalidation_file="last_execution.txt", regex_filename="2023_spotify_ds*.csv",
                      top_tracks_save_percentile=0.03, miner=miner, rules_mode="pairs")
    return job.run(cfg), base


def make_queries(base: pathlib.Path, n: int, seed: int = 0) -> List[List[str]]:
    from ..serve.index import RuleIndexData
    idx = RuleIndexData.load(base / "pickles" / "rules.idx")
    keys = [idx.names[i] for i in np.nonzero(idx.is_key)[0]]
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        k = int(rng.integers(1, 6))
        q = [keys[int(i)] for i in rng.integers(0, len(keys), k)]
        if rng.random() < 0.2:
            q = [f"unknown song {int(rng.integers(1e9))}"]
        out.append(q)
    return out


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def start_server(base: pathlib.Path, backend: str, workers: int, port: int,
                 front: str = "native", threads: int = 4, poll_minutes: float = 60.0):
    env = dict(os.environ)
    env.update(BASE_DIR=str(base) + "/", PICKLE_DIR="pickles/", SERVE_BACKEND=backend,
               KMLS_LOG_LEVEL="ERROR", POLLING_WAIT_IN_MINUTES=str(poll_minutes),
               PYTHONPATH=str(ROOT) + os.pathsep + env.get("PYTHONPATH", ""))
    cmd = [sys.executable, "-m", "kubernetes_machine_learning_server_amd.serve", "--host",
           "127.0.0.1", "--port", str(port), "--front", front, "--threads", str(threads),
           "--workers", str(workers), "--log-level", "error"]
    proc = subprocess.Popen(cmd, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE,
                            start_new_session=True)
    import urllib.request
    t0 = time.time()
    while time.time() - t0 < 240:
        if proc.poll() is not None:
            raise RuntimeError("server died: " + proc.stderr.read().decode()[-2000:])
        try:
            with urllib.request.urlopen(f"http://127.0.0.1:{port}/readyz", timeout=2) as r:
                if r.status == 200:
                    return proc
        except Exception:
            time.sleep(0.5)
    stop_server(proc)
    raise RuntimeError("server not ready after 240 s")


def stop_server(proc):
    try:
        os.killpg(proc.pid, signal.SIGTERM)
        proc.wait(timeout=20)
    except Exception:
        try:
            os.killpg(proc.pid, signal.SIGKILL)
        except Exception:
            pass


def _client(port: int, qps: float, duration: float, queries, t_start: float, out_q):
    import aiohttp

    async def run():
        lat, errs = [], 0
        conn = aiohttp.TCPConnector(limit=0, force_close=False)
        timeout = aiohttp.ClientTimeout(total=30)
        async with aiohttp.ClientSession(connector=conn, timeout=timeout) as sess:
            url = f"http://127.0.0.1:{port}/api/recommend/"
            n = int(qps * duration)
            tasks = []

            async def one(i, when):
                nonlocal errs
                await asyncio.sleep(max(0.0, when - time.perf_counter()))
                t = time.perf_counter()
                try:
                    async with sess.post(url, json={"songs": queries[i % len(queries)]}) as r:
                        await r.read()
                        if r.status != 200:
                            errs += 1
                            return
                except Exception:
                    errs += 1
                    return
                lat.append((time.perf_counter() - t, t - when))
            base = time.perf_counter() + max(0.0, t_start - time.time())
            for i in range(n):
                tasks.append(asyncio.ensure_future(one(i, base + i / qps)))
            await asyncio.gather(*tasks)
        return lat, errs
    lat, errs = asyncio.run(run())
    out_q.put((lat, errs))


def request_bytes(queries, port: int) -> List[bytes]:
    """Complete HTTP/1.1 requests for the native load generator (keep-alive)."""
    out = []
    for q in queries:
        body = json.dumps({"songs": q}, ensure_ascii=False).encode("utf-8")
        out.append(b"POST /api/recommend/ HTTP/1.1\r\nhost: 127.0.0.1:%d\r\n"
                   b"content-type: application/json\r\ncontent-length: %d\r\n\r\n"
                   % (port, len(body)) + body)
    return out


def measure_native(port: int, qps: float, duration: float, queries, connections: int = 64,
                   threads: int = 2) -> dict:
    from ..ops import native
    N = native.load()
    r = N.loadgen("127.0.0.1", port, request_bytes(queries, port), float(qps), float(duration),
                  connections, threads, 5.0)
    a = np.asarray(r["lat_ns"], np.float64) / 1e6
    lag = np.asarray(r["lag_ns"], np.float64) / 1e6
    if len(a) == 0:
        a = lag = np.full(1, np.inf)
    unanswered = int(r["offered"] - r["completed"])
    return {"offered_qps": qps, "completed": int(r["completed"]), "errors": int(r["errors"]),
            "unanswered": unanswered, "achieved_qps": round(r["completed"] / duration, 1),
            "p50_ms": round(float(np.percentile(a, 50)), 3),
            "p90_ms": round(float(np.percentile(a, 90)), 3),
            "p99_ms": round(float(np.percentile(a, 99)), 3),
            "p999_ms": round(float(np.percentile(a, 99.9)), 3),
            "max_ms": round(float(a.max()), 3), "mean_ms": round(float(a.mean()), 3),
            "send_lag_p99_ms": round(float(np.percentile(lag, 99)), 3),
            "latency_from": "scheduled send time", "connections": connections}


def _window(a: np.ndarray) -> dict:
    if len(a) == 0:
        return {"n": 0}
    return {"n": int(len(a)), "p50_ms": round(float(np.percentile(a, 50)), 3),
            "p99_ms": round(float(np.percentile(a, 99)), 3),
            "max_ms": round(float(a.max()), 3)}


def reload_under_load(port: int, base: pathlib.Path, alt_index: pathlib.Path, qps: float,
                      duration: float, reload_at: float, queries, connections: int = 64,
                      settle_s: float = 2.0) -> dict:
    """Open-loop load at `qps` for `duration` s; at `reload_at` s the job's publish step is
    replayed on the PVC (the alternate rules.idx renamed over the served one, then a new marker,
    written last), so the server's poller hot-reloads mid-run.  Latency percentiles (from the
    scheduled send time) before the flip, in the `settle_s` window after it, and after that."""
    import threading
    from ..ops import native
    from ..utils.atomic_io import atomic_write_bytes
    N = native.load()
    pk = base / "pickles"
    marker = base / "last_execution.txt"
    flip = {}

    def publisher():
        time.sleep(reload_at + 0.02)  # the load generator's clock starts 20 ms after connect
        t = time.time()
        atomic_write_bytes(pk / "rules.idx", alt_index.read_bytes())
        atomic_write_bytes(marker, f"reload-under-load {t:.3f}".encode())
        flip["t"] = time.time()

    th = threading.Thread(target=publisher, daemon=True)
    reloads0 = _metric(port, "kmls_reload_count")
    th.start()
    r = N.loadgen("127.0.0.1", port, request_bytes(queries, port), float(qps), float(duration),
                  connections, 2, 5.0)
    th.join()
    lat = np.asarray(r["lat_ns"], np.float64) / 1e6
    at = np.asarray(r["at_ns"], np.float64) / 1e9
    t1 = reload_at
    out = {"offered_qps": qps, "duration_s": duration, "reload_at_s": reload_at,
           "completed": int(r["completed"]), "errors": int(r["errors"]),
           "unanswered": int(r["offered"] - r["completed"]),
           "before": _window(lat[at < t1]),
           "during": _window(lat[(at >= t1) & (at < t1 + settle_s)]),
           "after": _window(lat[at >= t1 + settle_s]),
           "reloads": (_metric(port, "kmls_reload_count") or 0) - (reloads0 or 0),
           "latency_from": "scheduled send time (open loop)"}
    return out


def _metric(port: int, name: str) -> Optional[float]:
    import urllib.request
    try:
        with urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=5) as r:
            for ln in r.read().decode().splitlines():
                if ln.startswith(name + " ") or ln.startswith(name + "{"):
                    return float(ln.split()[-1])
    except Exception:
        return None
    return None


def capacity(port: int, queries, start_qps: float = 10000.0, duration: float = 2.0,
             p99_ms: float = 5.0, max_qps: float = 400000.0, connections: int = 128,
             threads: int = 2) -> dict:
    """Highest offered QPS answered with p99 < p99_ms (from scheduled time) and no errors:
    doubling from start_qps, then two bisection steps."""
    ok_q, ok_r, bad_q, trail = None, None, None, []

    def good(r):
        return r["errors"] == 0 and r["unanswered"] == 0 and r["p99_ms"] < p99_ms

    q = start_qps
    while q <= max_qps:
        r = measure_native(port, q, duration, queries, connections, threads)
        trail.append({k: r[k] for k in ("offered_qps", "achieved_qps", "p50_ms", "p99_ms",
                                        "errors", "unanswered")})
        if good(r):
            ok_q, ok_r = q, r
            q *= 2
        else:
            bad_q = q
            break
    if ok_q is not None and bad_q is not None:
        for _ in range(2):
            mid = (ok_q + bad_q) / 2
            r = measure_native(port, mid, duration, queries, connections, threads)
            trail.append({k: r[k] for k in ("offered_qps", "achieved_qps", "p50_ms", "p99_ms",
                                            "errors", "unanswered")})
            if good(r):
                ok_q, ok_r = mid, r
            else:
                bad_q = mid
    return {"max_qps_p99_under_ms": p99_ms, "capacity_qps": ok_q,
            "at_capacity": ok_r and {k: ok_r[k] for k in ("p50_ms", "p99_ms", "achieved_qps")},
            "limit_hit": bad_q is None, "trail": trail}


def cpu_info(server_pid: Optional[int] = None) -> dict:
    out = {"os_cpu_count": os.cpu_count()}
    try:
        out["affinity_cpus"] = len(os.sched_getaffinity(0))
    except Exception:
        pass
    if server_pid:
        try:
            import psutil
            p = psutil.Process(server_pid)
            t = p.cpu_times()
            out["server_cpu_s"] = round(t.user + t.system, 3)
            out["server_threads"] = p.num_threads()
        except Exception:
            pass
    t = os.times()
    out["bench_cpu_s"] = round(t.user + t.system, 3)
    return out


def measure(port: int, qps: float, duration: float, clients: int, queries) -> dict:
    ctx = mp.get_context("fork")
    q = ctx.Queue()
    t_start = time.time() + 1.0
    procs = [ctx.Process(target=_client, args=(port, qps / clients, duration,
                                                queries[c::clients], t_start, q))
             for c in range(clients)]
    for p in procs:
        p.start()
    lat, errs = [], 0
    for _ in procs:
        l, e = q.get(timeout=duration + 120)
        lat.extend(l)
        errs += e
    for p in procs:
        p.join(timeout=30)
    a = np.array([x[0] for x in lat]) * 1e3 if lat else np.zeros(1)
    lag = np.array([x[1] for x in lat]) * 1e3 if lat else np.zeros(1)
    return {"offered_qps": qps, "completed": len(lat), "errors": errs,
            "achieved_qps": round(len(lat) / duration, 1),
            "p50_ms": round(float(np.percentile(a, 50)), 3), "p90_ms": round(float(np.percentile(a, 90)), 3),
            "p99_ms": round(float(np.percentile(a, 99)), 3), "mean_ms": round(float(a.mean()), 3),
            "client_send_lag_p99_ms": round(float(np.percentile(lag, 99)), 3)}


def matcher_bench(base: pathlib.Path, n_queries: int = 20000) -> dict:
    """In-process matcher throughput (no HTTP): python reference vs C++ vs HIP batched."""
    from ..models.oracle import recommend_oracle
    from ..ops import native
    from ..serve.index import RuleIndexData
    idx = RuleIndexData.load(base / "pickles" / "rules.idx")
    rec = idx.to_rec_dict()
    qs = make_queries(base, n_queries, seed=1)
    n2i = idx.name_to_id
    ids = [np.array([n2i.get(s, -1) for s in q], np.int32) for q in qs]
    q_ptr = np.zeros(len(ids) + 1, np.int64)
    np.cumsum([len(x) for x in ids], out=q_ptr[1:])
    seeds = np.concatenate(ids)
    out = {"n_queries": n_queries, "index_keys": idx.n_keys, "index_nnz": idx.nnz}
    t = time.perf_counter()
    for q in qs[:5000]:
        recommend_oracle(rec, q, 10)
    out["python_ref_us_per_query"] = round((time.perf_counter() - t) / 5000 * 1e6, 2)
    host = idx.native()
    t = time.perf_counter()
    for x in ids:
        host.query(x, 10)
    out["cpp_single_us_per_query"] = round((time.perf_counter() - t) / len(ids) * 1e6, 3)
    t = time.perf_counter()
    host.query_batch(q_ptr, seeds, 10)
    out["cpp_batch_us_per_query"] = round((time.perf_counter() - t) / len(ids) * 1e6, 3)
    if native.gpu_available():
        N = native.load()
        g = N.GpuRuleIndex(0, host)
        for B in (1, 16, 256, 4096, n_queries):
            qp = q_ptr[:B + 1]
            sd = seeds[:qp[-1]]
            g.query_batch(qp, sd, 10)  # warm
            reps = max(3, 2000 // B)
            t = time.perf_counter()
            for _ in range(reps):
                r_ids, r_n = g.query_batch(qp, sd, 10)
            dt = (time.perf_counter() - t) / reps
            c_ids, c_n = host.query_batch(qp, sd, 10)
            out[f"hip_batch{B}_us_per_batch"] = round(dt * 1e6, 2)
            out[f"hip_batch{B}_us_per_query"] = round(dt / B * 1e6, 3)
            out[f"hip_batch{B}_exact"] = bool((r_ids == c_ids).all() and (r_n == c_n).all())
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", default="auto", help="hip | loop | cpu | python | auto")
    ap.add_argument("--qps", default="2000,5000,10000")
    ap.add_argument("--duration", type=float, default=5.0)
    ap.add_argument("--front", choices=("native", "uvicorn"), default="native")
    ap.add_argument("--threads", type=int, default=4, help="native front I/O threads")
    ap.add_argument("--workers", type=int, default=4, help="uvicorn front workers")
    ap.add_argument("--client", choices=("native", "python"), default="native")
    ap.add_argument("--clients", type=int, default=8, help="python client processes")
    ap.add_argument("--connections", type=int, default=64)
    ap.add_argument("--capacity", action="store_true", help="find the max QPS with p99 < 5 ms")
    ap.add_argument("--json-out", default=None, help="also write the summary JSON here")
    ap.add_argument("--matcher-only", action="store_true")
    ap.add_argument("--pvc", default=None, help="reuse a populated PVC dir")
    ap.add_argument("--reload-index", default=None,
                    help="rules.idx to hot-swap in mid-run (reload under load)")
    ap.add_argument("--reload-at", type=float, default=4.0)
    ap.add_argument("--reload-qps", type=float, default=10000.0)
    ap.add_argument("--reload-duration", type=float, default=10.0)
    ap.add_argument("--poll-minutes", type=float, default=0.01,
                    help="server marker poll interval for --reload-index (POLLING_WAIT_IN_MINUTES)")
    a = ap.parse_args(argv)
    tmp = tempfile.mkdtemp(prefix="kmls_serve_") if a.pvc is None else a.pvc
    root = pathlib.Path(tmp)
    if not (root / "api-data" / "pickles" / "rules.idx").exists():
        summary, base = prepare_pvc(root)
    base = root / "api-data"
    if a.matcher_only:
        print(json.dumps({"bench": "matcher", **matcher_bench(base)}), flush=True)
        return 0
    reload = None
    if a.reload_index:
        reload = {"alt_index": a.reload_index, "at": a.reload_at, "qps": a.reload_qps,
                  "duration": a.reload_duration, "poll_minutes": a.poll_minutes}
    summary = run_serve_bench(base, a.backend, [float(x) for x in a.qps.split(",") if x],
                              a.duration, a.front, a.threads, a.workers, a.client, a.clients,
                              a.connections, a.capacity, verbose=True, reload=reload)
    print(json.dumps({"bench": "serve_summary", **summary}), flush=True)
    if a.json_out:
        pathlib.Path(a.json_out).write_text(json.dumps(summary))
    return 0


def run_serve_bench(base: pathlib.Path, backend: str, qps_list, duration: float,
                    front: str = "native", threads: int = 4, workers: int = 4,
                    client: str = "native", clients: int = 8, connections: int = 64,
                    with_capacity: bool = True, verbose: bool = False,
                    reload: Optional[dict] = None) -> dict:
    """Start the server (a fresh child process), run the fixed-QPS points and the capacity
    search, stop the server.  Returns the summary dict (bench.py's ``serve`` block)."""
    queries = make_queries(base, 50000)
    port = _free_port()
    t_start = time.time()
    proc = start_server(base, backend, workers, port, front=front, threads=threads,
                        poll_minutes=(reload or {}).get("poll_minutes", 60.0))
    res = {"backend": backend, "front": front,
           "threads" if front == "native" else "workers": threads if front == "native" else workers,
           "client": client, "duration_s": duration, "points": []}
    try:
        import urllib.request
        with urllib.request.urlopen(f"http://127.0.0.1:{port}/readyz", timeout=5) as r:
            ready = json.loads(r.read())
        res["server_ready_s"] = round(time.time() - t_start, 2)
        res["gpu_index"] = ready.get("gpu_index")
        res["gpu_min_batch"] = ready.get("gpu_min_batch")
        res["crossover_us"] = ready.get("crossover_us")
        res["gpu_min_merge"] = ready.get("gpu_min_merge")
        res["loop_crossover_us"] = ready.get("loop_crossover_us")
        if verbose:
            print(json.dumps({"bench": "serve_ready", **{k: res[k] for k in
                  ("backend", "gpu_index", "gpu_min_batch", "crossover_us", "gpu_min_merge",
                   "loop_crossover_us")}}), flush=True)
        # warm-up
        if client == "native":
            measure_native(port, 500, 1.0, queries, connections)
        else:
            measure(port, 200, 1.0, 1, queries)
        for qps in qps_list:
            if client == "native":
                r = measure_native(port, qps, duration, queries, connections)
            else:
                r = measure(port, qps, duration, clients, queries)
            res["points"].append(r)
            if verbose:
                print(json.dumps({"bench": "serve", **r}), flush=True)
        if reload:
            res["reload_under_load"] = reload_under_load(
                port, base, pathlib.Path(reload["alt_index"]), reload["qps"], reload["duration"],
                reload["at"], queries, connections)
            if verbose:
                print(json.dumps({"bench": "reload_under_load", **res["reload_under_load"]}),
                      flush=True)
        if with_capacity and client == "native":
            res["capacity"] = capacity(port, queries, start_qps=max(qps_list or [10000.0]) * 2)
            if verbose:
                print(json.dumps({"bench": "capacity", **res["capacity"]}), flush=True)
        try:
            with urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=5) as r:
                m = r.read().decode()
            res["front_stats"] = {ln.split()[0][len("kmls_front_"):]: int(float(ln.split()[1]))
                                  for ln in m.splitlines() if ln.startswith("kmls_front_")}
        except Exception:
            pass
        res["cpu"] = cpu_info(proc.pid)
    finally:
        stop_server(proc)
    return res


if __name__ == "__main__":
    sys.exit(main())
