"""FastAPI recommendation server (HTTP surface §2.H).

Compatible with ``rest_api/app/main.py``: same title/summary/version/tags, the same
``POST /api/recommend/`` schema and its three OpenAPI examples (``normal``, ``uncommon``,
``absent``), ``GET /`` HTML client, ``GET /test`` redirect, ``/static`` mount, response
``{"songs", "model_date", "version"}``, 400 on an empty list, the same log lines and the same
env vars.  New: ``/healthz`` (liveness), ``/readyz`` (index loaded), ``/metrics``
(Prometheus), HBM-resident rule index + micro-batched HIP matcher (``SERVE_BACKEND=hip``).

Run: ``uvicorn kubernetes_machine_learning_server_amd.serve.app:app --port 80``
(or ``python -m kubernetes_machine_learning_server_amd.serve``).
"""
from __future__ import annotations

import asyncio
import contextlib
import logging
import os
import random
import sys
import time
from typing import Annotated, List, Optional

from fastapi import Body, FastAPI, HTTPException, Request
from fastapi.responses import HTMLResponse, JSONResponse, PlainTextResponse, RedirectResponse
from fastapi.staticfiles import StaticFiles
from fastapi.templating import Jinja2Templates
from pydantic import BaseModel

from ..config import ApiSettings
from . import matcher as M
from .batcher import MicroBatcher
from .state import ReloadManager

logger = logging.getLogger("kmls.api")


def _setup_logging() -> None:
    if getattr(_setup_logging, "_done", False):
        return
    logger.setLevel(os.environ.get("KMLS_LOG_LEVEL", "DEBUG").upper())
    h = logging.StreamHandler(sys.stdout)
    h.setFormatter(logging.Formatter(fmt="%(asctime)s - %(levelname)s - %(message)s"))
    logger.addHandler(h)
    logger.propagate = False
    _setup_logging._done = True


class SongRequest(BaseModel):
    songs: List[str]


OPENAPI_EXAMPLES = {
    "normal": {
        "summary": "Common songs",
        "description": "Will give normal recommendations",
        "value": {"songs": ["Gold Digger", "Closer"]},
    },
    "uncommon": {
        "summary": "Songs not that common",
        "value": {"songs": ["The Motto", "Despacito"]},
    },
    "absent": {
        "summary": "Songs without recommendations",
        "value": {"songs": ["Evidencias", "Esse cara sou eu"]},
    },
}

TAGS_METADATA = [{"name": "recommend", "description": "Song recommendation service"}]


def _python_match(snap, seeds, k):
    rec = getattr(snap, "_py_rec", None)
    if rec is None:
        rec = snap.index.to_rec_dict()
        object.__setattr__(snap, "_py_rec", rec)
    from ..models.oracle import recommend_oracle
    return recommend_oracle(rec, seeds, k)


def _gpu_factory(cfg: ApiSettings):
    """HBM index builder for SERVE_BACKEND=hip|auto (None → CPU matcher only).  The GPU serving
    process is the native front (serve/front.py: one process, the HIP matcher micro-batched
    across its I/O threads in-process); uvicorn workers of the multi-process runner stay on the
    C++ matcher (KMLS_NO_GPU=1 is set for them), so no two processes share one card's index."""
    if cfg.serve_backend in ("cpu", "python") or os.environ.get("KMLS_NO_GPU") == "1":
        return None
    from ..ops import native
    if not native.gpu_available():
        if cfg.serve_backend in ("hip", "loop"):
            raise RuntimeError(f"SERVE_BACKEND={cfg.serve_backend} but no HIP device is visible")
        return None
    N = native.load()
    dev = int(os.environ.get("KMLS_DEVICE", "0"))

    def build(index):
        return N.GpuRuleIndex(dev, index.native())
    return build


class _Metrics:
    def __init__(self):
        from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram
        self.registry = CollectorRegistry()
        self.requests = Counter("kmls_recommend_requests_total", "recommend requests",
                                ["outcome"], registry=self.registry)
        self.latency = Histogram("kmls_recommend_latency_seconds", "server-side latency",
                                 buckets=(1e-5, 3e-5, 1e-4, 3e-4, 1e-3, 3e-3, 1e-2, 3e-2, 0.1, 1.0),
                                 registry=self.registry)
        self.reloads = Gauge("kmls_reload_count", "successful reloads", registry=self.registry)
        self.keys = Gauge("kmls_index_keys", "rule-index keys", registry=self.registry)
        self.nnz = Gauge("kmls_index_nnz", "rule-index entries", registry=self.registry)
        self.batch = Gauge("kmls_last_batch_size", "last matcher batch", registry=self.registry)
        self.gpu_batches = Gauge("kmls_gpu_batches", "batches answered by the HIP kernel",
                                 registry=self.registry)


def create_app(cfg: Optional[ApiSettings] = None, native_front: bool = False) -> FastAPI:
    """``native_front``: the app sits behind serve/front.py, which answers the hot route itself
    (and owns the GPU batching); requests that reach this app's route are the rare ones the
    front hands over, answered here by the C++ matcher."""
    cfg = cfg or ApiSettings.from_env()
    _setup_logging()
    logger.info("API is starting up")
    logger.info(f"Will search for templates on {cfg.templates_dir}")
    mgr = ReloadManager(cfg, gpu_factory=_gpu_factory(cfg))
    batcher = MicroBatcher(cfg.batch_max, cfg.batch_wait_us, cfg.gpu_min_batch)
    metrics = _Metrics()
    period = max(1.0, 60.0 * cfg.polling_wait_in_minutes)

    async def poll_loop():
        # repeat_every(seconds=60*POLLING_WAIT_IN_MINUTES): the first tick runs at startup
        while True:
            await asyncio.sleep(period)
            try:
                await asyncio.to_thread(mgr.reload_data_if_required)
            except Exception as e:  # pragma: no cover
                logger.error(f"reload tick failed: {e}")

    @contextlib.asynccontextmanager
    async def lifespan(app: FastAPI):
        await asyncio.to_thread(mgr.reload_data_if_required)
        batcher.start()
        task = asyncio.get_running_loop().create_task(poll_loop())
        try:
            yield
        finally:
            task.cancel()
            await batcher.stop()
            logger.info("Exiting...")

    app = FastAPI(title="Music Recommendation API", version=cfg.version,
                  summary="Kubernetes based deployment with fpgrowth recommendations",
                  openapi_tags=TAGS_METADATA, lifespan=lifespan)
    static_dir = cfg.static_dir
    static_dir.mkdir(parents=True, exist_ok=True)  # the reference crashes if it is missing
    app.mount("/static", StaticFiles(directory=str(static_dir)), name="static")
    templates = Jinja2Templates(directory=str(cfg.templates_dir))
    app.state.mgr = mgr
    app.state.cfg = cfg
    app.state.batcher = batcher
    app.state.metrics = metrics
    app.state.front = None  # serve/front.py sets its _native.HttpFront here

    @app.get("/test", tags=["util"], include_in_schema=False)
    def redirect_to_doc():
        return RedirectResponse(url="/docs#/recommend/get_recommendations_api_recommend__post")

    async def recommend_tracks_for_track(seeds: List[str]) -> List[str]:
        snap = mgr.snapshot
        if snap is None:
            logger.error("Recommendations not loaded, calling pickle reload")
            asyncio.get_running_loop().run_in_executor(None, mgr.reload_data_if_required)
            metrics.requests.labels("not_loaded").inc()
            return [M.NO_RECOMMENDATIONS]
        k = cfg.k_best_tracks
        if cfg.serve_backend == "python":
            # the reference's own matcher (dict-of-dicts + defaultdict + sorted), for A/B benches
            res = _python_match(snap, seeds, k)
        elif (not native_front and snap.gpu_index is not None and snap.gpu_min_batch is not None
              and inflight[0] >= batcher._gpu_min(snap)):
            # enough requests in flight to fill a batch the HIP matcher answers faster (the
            # crossover measured on this index): queue for the micro-batcher.  Below that the
            # queue hop would only add latency, so the C++ matcher answers inline.
            ids, n = await batcher.submit(snap, M.seed_ids(snap, seeds), k)
            res = None if n < 0 else [snap.index.names[i] for i in ids[:n]]
            metrics.batch.set(batcher.last_batch)
            metrics.gpu_batches.set(batcher.gpu_batches)
        else:
            res = M.recommend_cpu(snap, seeds, k)
        if res is None:
            logger.warning(f"Tracks [{seeds}] not found in the song recommendation list.")
            metrics.requests.labels("fallback").inc()
            return M.static_recommendation(snap, seeds, k)
        metrics.requests.labels("rules").inc()
        return res

    inflight = [0]  # requests of this worker between validation and response

    @app.post("/api/recommend/", tags=["recommend"])
    async def get_recommendations(request: Annotated[SongRequest, Body(openapi_examples=OPENAPI_EXAMPLES)]):
        t0 = time.perf_counter()
        if not request.songs:
            metrics.requests.labels("empty").inc()
            raise HTTPException(status_code=400, detail="The songs list cannot be empty.")
        inflight[0] += 1
        try:
            songs = await recommend_tracks_for_track(request.songs)
        finally:
            inflight[0] -= 1
        metrics.latency.observe(time.perf_counter() - t0)
        return {"songs": songs, "model_date": mgr.cache_value, "version": cfg.version}

    @app.get("/", response_class=HTMLResponse, include_in_schema=False)
    async def render_client(request: Request):
        if mgr.snapshot is None:
            logger.info("Best tracks not loaded, waiting for data to be loaded")
            await asyncio.sleep(2)
        snap = mgr.snapshot
        if snap is None or not snap.best_tracks:
            logger.error("Best tracks not loaded")
            return HTMLResponse("Recommendations model not loaded yet", status_code=503)
        seed_track = random.choice(snap.best_tracks)["track_name"]
        tracks = M.static_recommendation(snap, [seed_track], cfg.k_best_tracks)
        return templates.TemplateResponse(request=request, name="client.html",
                                          context={"tracks": tracks})

    @app.get("/healthz", include_in_schema=False)
    def healthz():
        return {"status": "ok"}

    @app.get("/readyz", include_in_schema=False)
    def readyz():
        snap = mgr.snapshot
        if snap is None:
            return JSONResponse({"ready": False, "error": mgr.last_error}, status_code=503)
        return {"ready": True, "model_date": snap.marker, "keys": snap.index.n_keys,
                "source": snap.source, "gpu_index": snap.gpu_index is not None,
                "gpu_min_batch": snap.gpu_min_batch,
                "crossover_us": {str(b): v for b, v in (snap.crossover or {}).items()},
                "gpu_min_merge": snap.gpu_min_merge,
                "loop_crossover_us": dict(snap.loop_crossover or {})}

    @app.get("/metrics", include_in_schema=False)
    def prometheus_metrics():
        from prometheus_client import generate_latest
        snap = mgr.snapshot
        metrics.reloads.set(mgr.reload_counter)
        if snap is not None:
            metrics.keys.set(snap.index.n_keys)
            metrics.nnz.set(snap.index.nnz)
        text = generate_latest(metrics.registry).decode()
        front = app.state.front
        if front is not None:  # the native front's own counters (its hot route bypasses this app)
            for k, v in front.stats().items():
                text += f"# TYPE kmls_front_{k} counter\nkmls_front_{k} {v}\n"
        return PlainTextResponse(text, media_type="text/plain; version=0.0.4")

    return app


def __getattr__(name):  # lazy module-level ``app`` for ``uvicorn ...serve.app:app``
    if name == "app":
        a = create_app()
        globals()["app"] = a
        return a
    raise AttributeError(name)
