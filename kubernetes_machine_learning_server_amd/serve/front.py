"""Native serving front runner: one process, C++ HTTP I/O threads, the FastAPI app behind them.

``python -m kubernetes_machine_learning_server_amd.serve --front native --threads 4``

* ``_native.HttpFront`` (csrc/host/http_front.cpp) owns the listening sockets (one per I/O
  thread, SO_REUSEPORT) and answers ``POST /api/recommend/`` natively from the current model
  generation: C++ matcher, or the HIP matcher over the HBM index micro-batched across all
  connections in-process (no GPU-owner process, no IPC), plus the static fallback.
* Everything else (``/``, ``/docs``, ``/openapi.json``, ``/test``, ``/healthz``, ``/readyz``,
  ``/metrics``, ``/static``, malformed or empty bodies, a not-yet-loaded model) is passed to the
  FastAPI app (``serve/app.py``) through an eventfd-signalled queue and run by this asyncio
  loop as a plain ASGI call, so those responses are FastAPI's own.
* The app's lifespan runs here as for uvicorn: initial load, the marker-polling hot reload.
  Every successful reload pushes the new snapshot into the front (atomic swap in C++).

The reference's equivalent stack is uvicorn + httptools + uvloop (C/Cython); those
are not available in this image, and pure-Python h11 caps a worker at a few thousand requests/s.
"""
from __future__ import annotations

import asyncio
import logging
import os
import signal
import urllib.parse
from typing import Any, List, Optional, Tuple

logger = logging.getLogger("kmls.api")


def _latin1(b) -> str:
    return b.decode("latin-1") if isinstance(b, (bytes, bytearray)) else str(b)


class NativeFront:
    def __init__(self, app, host: str = "0.0.0.0", port: int = 80, threads: int = 4):
        from ..ops import native
        self.app = app
        self.cfg = app.state.cfg
        self.N = native.load()
        self.host, self.port_req, self.threads = host, port, max(1, int(threads))
        self.front = self.N.HttpFront(host, port, self.threads, self.cfg.k_best_tracks,
                                      self.cfg.version, self.cfg.batch_max,
                                      self.cfg.batch_wait_us)
        self.state: dict = {}
        self._tasks: set = set()
        app.state.front = self.front

    # -- model push ---------------------------------------------------------------------------
    def push(self, snap) -> None:
        idx = snap.index
        names = list(idx.names) if idx.names is not None else [str(i) for i in range(idx.n_items)]
        gpu = snap.gpu_index if (snap.gpu_index is not None and
                                 isinstance(snap.gpu_index, self.N.GpuRuleIndex)) else None
        gmm = getattr(snap, "gpu_min_merge", None)
        self.front.set_model(idx.native(), names, snap.best_track_names, snap.marker, gpu,
                             int(snap.gpu_min_batch or 0) if gpu is not None else 0,
                             int(gmm) if (gpu is not None and gmm is not None) else -1)

    # -- ASGI bridge for the slow path ----------------------------------------------------------
    def _drain(self) -> None:
        while True:
            r = self.front.next_slow()
            if r is None:
                return
            t = asyncio.get_running_loop().create_task(self._handle(r))
            self._tasks.add(t)
            t.add_done_callback(self._tasks.discard)

    async def _handle(self, r: Tuple) -> None:
        token, method, path, query, http_version, headers, body, chost, cport = r
        status, out_headers, chunks = 500, [], []
        try:
            scope = {
                "type": "http", "asgi": {"version": "3.0", "spec_version": "2.3"},
                "http_version": http_version, "method": method, "scheme": "http",
                "path": urllib.parse.unquote(path.decode("latin-1")), "raw_path": path,
                "query_string": query, "root_path": "", "headers": list(headers),
                "client": (chost, cport), "server": (self.host, self.front.port),
                "state": dict(self.state),
            }
            sent = [False]
            done = asyncio.Event()

            async def receive():
                if not sent[0]:
                    sent[0] = True
                    return {"type": "http.request", "body": body, "more_body": False}
                await done.wait()
                return {"type": "http.disconnect"}

            async def send(msg):
                nonlocal status, out_headers
                if msg["type"] == "http.response.start":
                    status = int(msg["status"])
                    out_headers = [(_latin1(k), _latin1(v)) for k, v in msg.get("headers", [])]
                elif msg["type"] == "http.response.body":
                    chunks.append(bytes(msg.get("body", b"")))
                    if not msg.get("more_body", False):
                        done.set()

            await self.app(scope, receive, send)
            done.set()
        except Exception as e:  # pragma: no cover - FastAPI turns handler errors into 500s itself
            logger.error(f"front: ASGI call failed: {e!r}")
            status, out_headers, chunks = 500, [("content-type", "text/plain; charset=utf-8")], \
                [b"Internal Server Error"]
        body_out = b"" if method == "HEAD" else b"".join(chunks)
        self.front.respond(token, status, out_headers, body_out)

    # -- lifespan -----------------------------------------------------------------------------
    async def _lifespan(self, phase: str, inbox: asyncio.Queue, outbox: asyncio.Queue) -> None:
        await inbox.put({"type": f"lifespan.{phase}"})
        msg = await outbox.get()
        if msg["type"].endswith(".failed"):
            raise RuntimeError(f"lifespan {phase} failed: {msg.get('message')}")

    async def serve(self, stop: Optional[asyncio.Event] = None) -> None:
        loop = asyncio.get_running_loop()
        stop = stop or asyncio.Event()
        inbox: asyncio.Queue = asyncio.Queue()
        outbox: asyncio.Queue = asyncio.Queue()
        life = loop.create_task(self.app({"type": "lifespan", "asgi": {"version": "3.0"},
                                          "state": self.state}, inbox.get, outbox.put))
        mgr = self.app.state.mgr
        mgr.listeners.append(self.push)
        await self._lifespan("startup", inbox, outbox)
        if mgr.snapshot is not None:  # loaded during startup (before the listener could fire)
            self.push(mgr.snapshot)
        loop.add_reader(self.front.slow_fd, self._drain)
        await asyncio.to_thread(self.front.start)
        logger.info(f"native front listening on {self.host}:{self.front.port} "
                    f"({self.threads} I/O threads)")
        try:
            await stop.wait()
        finally:
            loop.remove_reader(self.front.slow_fd)
            await asyncio.to_thread(self.front.stop)
            await self._lifespan("shutdown", inbox, outbox)
            life.cancel()


def run_native(host: str = "0.0.0.0", port: int = 80, threads: int = 4) -> int:
    os.environ.setdefault("KMLS_NATIVE_FRONT", "1")
    from .app import create_app
    app = create_app(native_front=True)
    front = NativeFront(app, host, port, threads)

    async def main():
        stop = asyncio.Event()
        loop = asyncio.get_running_loop()
        for sig in (signal.SIGTERM, signal.SIGINT):
            loop.add_signal_handler(sig, stop.set)
        await front.serve(stop)

    asyncio.run(main())
    return 0
