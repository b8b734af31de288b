"""Multi-process server launcher: one SO_REUSEPORT socket per worker process.

uvicorn's own ``--workers N`` mode binds the socket in the supervisor and hands the fd to the
workers; the inherited socket object reports ``proto == 0``, so asyncio's transport never sets
TCP_NODELAY on accepted connections and every response pays Nagle + the client's 40 ms delayed
ACK (measured: p50 44 ms at 500 QPS vs 1 ms with one worker).  Here each worker creates its own
``socket(AF_INET, SOCK_STREAM, IPPROTO_TCP)`` with SO_REUSEPORT on the same port — the kernel
load-balances connections across workers and NODELAY is applied — and serves it with
``uvicorn.Server``.  Each worker is a full app instance (its own model snapshot / HBM index).
"""
from __future__ import annotations

import multiprocessing as mp
import os
import signal
import socket
import sys
import time
from typing import List


def make_socket(host: str, port: int, reuse_port: bool) -> socket.socket:
    fam = socket.AF_INET6 if ":" in host else socket.AF_INET
    s = socket.socket(fam, socket.SOCK_STREAM, socket.IPPROTO_TCP)
    s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    if reuse_port:
        s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEPORT, 1)
    s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
    s.bind((host, port))
    s.listen(2048)
    s.setblocking(False)
    return s


def _worker(host: str, port: int, reuse_port: bool, log_level: str) -> None:
    import uvicorn
    sock = make_socket(host, port, reuse_port)
    cfg = uvicorn.Config("kubernetes_machine_learning_server_amd.serve.app:app", log_level=log_level,
                         access_log=False, lifespan="on", backlog=2048)
    server = uvicorn.Server(cfg)
    server.run(sockets=[sock])


def _owner(path: str) -> None:
    from .gpu_owner import owner_main
    sys.exit(owner_main(path))


def _start_owner(ctx, workers: int):
    """The GPU-owning matcher process (serve/gpu_owner.py) for multi-worker GPU serving: started
    first; workers find its socket through KMLS_GPU_OWNER_SOCKET.  This launcher never touches
    the GPU itself (a process that has initialised HIP must not fork+exec workers)."""
    backend = os.environ.get("SERVE_BACKEND", "auto").lower()
    if workers <= 1 or backend not in ("auto", "hip") or os.environ.get("KMLS_GPU_OWNER") == "0":
        return None
    path = os.environ.get("KMLS_GPU_OWNER_SOCKET") or f"/tmp/kmls_gpu_owner_{os.getpid()}.sock"
    os.environ["KMLS_GPU_OWNER_SOCKET"] = path
    p = ctx.Process(target=_owner, args=(path,), daemon=False)
    p.start()
    deadline = time.time() + float(os.environ.get("KMLS_GPU_OWNER_WAIT_S", "180"))
    while time.time() < deadline and p.is_alive() and not os.path.exists(path):
        time.sleep(0.1)
    return p


def run(host: str = "0.0.0.0", port: int = 80, workers: int = 1, log_level: str = "info") -> int:
    if workers <= 1:
        _worker(host, port, False, log_level)
        return 0
    ctx = mp.get_context("spawn")
    owner = _start_owner(ctx, workers)
    procs: List[mp.Process] = [ctx.Process(target=_worker, args=(host, port, True, log_level),
                                           daemon=False) for _ in range(workers)]
    for p in procs:
        p.start()
    if owner is not None:
        procs.append(owner)

    def stop(signum, frame):
        for p in procs:
            if p.is_alive():
                os.kill(p.pid, signal.SIGTERM)

    signal.signal(signal.SIGTERM, stop)
    signal.signal(signal.SIGINT, stop)
    rc = 0
    try:
        while any(p.is_alive() for p in procs):
            for p in procs:
                p.join(timeout=0.5)
                if p.exitcode not in (None, 0):
                    rc = p.exitcode
    finally:
        stop(None, None)
        for p in procs:
            p.join(timeout=10)
    return rc
