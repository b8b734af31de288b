"""Server launchers.

* ``native`` (default): serve/front.py — one process, C++ HTTP I/O threads, the FastAPI app
  behind them for every route the front does not answer itself, GPU matching in-process.
* ``uvicorn``: the pure FastAPI/uvicorn stack (the reference's own serving stack),
  ``workers`` processes.  uvicorn's own ``--workers N`` mode binds the socket in the supervisor
  and hands the fd to the workers; the inherited socket object reports ``proto == 0``, so
  asyncio's transport never sets TCP_NODELAY on accepted connections and every response pays
  Nagle + the client's 40 ms delayed ACK.  Here each worker creates its own
  ``socket(AF_INET, SOCK_STREAM, IPPROTO_TCP)`` with SO_REUSEPORT on the same port — the kernel
  load-balances connections and NODELAY is applied.  Multi-worker uvicorn stays on the C++
  matcher (the GPU belongs to one process: use the native front for HIP serving).
"""
from __future__ import annotations

import multiprocessing as mp
import os
import signal
import socket
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


def run(host: str = "0.0.0.0", port: int = 80, workers: int = 1, log_level: str = "info") -> int:
    """uvicorn front (``--front uvicorn``)."""
    if workers <= 1:
        _worker(host, port, False, log_level)
        return 0
    os.environ["KMLS_NO_GPU"] = "1"  # inherited by the spawned workers
    ctx = mp.get_context("spawn")
    procs: List[mp.Process] = [ctx.Process(target=_worker, args=(host, port, True, log_level),
                                           daemon=False) for _ in range(workers)]
    for p in procs:
        p.start()

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
