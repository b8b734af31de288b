"""Model state and hot reload (reference ``rest_api/app/main.py:52-122``).

Protocol kept: poll the marker ``last_execution.txt`` every ``POLLING_WAIT_IN_MINUTES``;
reload when it changed or when nothing is loaded yet; ``model_date`` = marker contents; the
same log lines (they are the reference's reload test oracle, ``relatorio.pdf`` p.7).

Fixes: the loaded model is ONE immutable snapshot object
swapped by a single reference assignment (no torn best_tracks/recommendations pair), the marker
value is committed only after a successful load (a failed reload is retried on the next tick
instead of being forgotten), and a missing artifact at boot does not crash the process — the
server stays up, reports not-ready, and keeps polling.
"""
from __future__ import annotations

import dataclasses
import logging
import pathlib
import pickle
import threading
import time
from typing import Any, Dict, List, Optional

import numpy as np

from ..config import ApiSettings
from .index import RuleIndexData

logger = logging.getLogger("kmls.api")

RULES_INDEX_FILE = "rules.idx"


@dataclasses.dataclass(frozen=True)
class ModelSnapshot:  # immutable; _py_rec (python backend cache) is set once via object.__setattr__
    best_tracks: List[Dict[str, Any]]
    index: RuleIndexData
    marker: Optional[str]
    loaded_at: float
    n_recommendations: int
    source: str  # "rules.idx" | "pickle"
    gpu_index: Any = None  # _native.GpuRuleIndex when SERVE_BACKEND uses the GPU
    # smallest batch the HIP matcher answers faster than the C++ one on THIS index (measured
    # when the snapshot is built; None = the GPU never wins, every batch stays on the CPU)
    gpu_min_batch: Optional[int] = None
    crossover: Any = None  # the measurement behind gpu_min_batch
    # persistent serving kernel: queries whose merged rows hold >= this many entries (up to the
    # wave matcher's 512) go to it one by one (None = off); and the measurement behind it
    gpu_min_merge: Optional[int] = None
    loop_crossover: Any = None

    @property
    def best_track_names(self) -> List[str]:
        return [t["track_name"] for t in self.best_tracks]


def read_pickle_dict(cfg: ApiSettings, prefer_index: bool = True):
    """Load best tracks + recommendations (``read_pickle_dict``, main.py:52-80).

    ``best_tracks.pickle`` is required (``ValueError`` otherwise, as the reference).  The rules
    come from ``rules.idx`` (binary CSR written by our job, no unpickling) when it is at least as
    new as ``recommendations.pickle``; otherwise from the pickle (any reference-format dict,
    e.g. one written by the reference job), indexed preserving its inner order.
    """
    cfg.base_dir.mkdir(parents=True, exist_ok=True)
    cfg.pickles_folder.mkdir(parents=True, exist_ok=True)
    best_path = cfg.pickles_folder / cfg.best_tracks_file
    if not best_path.exists():
        logger.error(f"Best tracks file not found at {best_path}")
        raise ValueError(f"Best tracks file not found at {best_path}")
    with open(best_path, "rb") as f:
        best_tracks = pickle.load(f)
    logger.info(f"Best tracks loaded: {len(best_tracks)}")
    rec_path = cfg.pickles_folder / cfg.recommendations_file
    idx_path = cfg.pickles_folder / RULES_INDEX_FILE
    use_idx = (prefer_index and idx_path.exists() and
               (not rec_path.exists() or idx_path.stat().st_mtime >= rec_path.stat().st_mtime))
    index = None
    if use_idx:
        try:
            index = RuleIndexData.load(idx_path)
            source = "rules.idx"
        except Exception as e:  # unreadable index: the pickle is the reference artifact
            logger.error(f"Rule index {idx_path} unreadable ({e!r}); falling back to the pickle")
            index = None
    if index is None:
        with open(rec_path, "rb") as f:
            rec = pickle.load(f)
        index = RuleIndexData.from_rec_dict(rec)
        source = "pickle"
    logger.info(f"Recommendations loaded: {index.n_keys}")
    return best_tracks, index, source


def measure_crossover(index, gpu_index, k: int = 10, reps: int = 5, seed: int = 0):
    """Time the C++ and HIP batch matchers on sample queries of this index (1-5 key seeds)
    for batch sizes 1..1024; returns (smallest batch where the GPU is faster, {B: (cpu_us,
    gpu_us)}).  The auto router (SERVE_BACKEND=auto) sends only batches at least that large to
    the GPU, so at loads that never build such batches the GPU is provably never used."""
    import numpy as np
    keys = np.nonzero(index.is_key)[0]
    if len(keys) == 0:
        return None, {}
    rng = np.random.default_rng(seed)
    host = index.native()
    res = {}
    best = None
    for B in (1, 4, 16, 64, 256, 1024):
        lens = rng.integers(1, 6, size=B)
        q_ptr = np.zeros(B + 1, np.int64)
        np.cumsum(lens, out=q_ptr[1:])
        seeds = keys[rng.integers(0, len(keys), int(q_ptr[-1]))].astype(np.int32)
        gpu_index.query_batch(q_ptr, seeds, k)  # warm
        tc, tg = [], []
        for _ in range(reps):
            t0 = time.perf_counter()
            host.query_batch(q_ptr, seeds, k)
            tc.append(time.perf_counter() - t0)
            t0 = time.perf_counter()
            gpu_index.query_batch(q_ptr, seeds, k)
            tg.append(time.perf_counter() - t0)
        c, g = float(np.median(tc)) * 1e6, float(np.median(tg)) * 1e6
        res[B] = (round(c, 2), round(g, 2))
        if best is None and g < c:
            best = B
    return best, res


MERGE_BINS = ((1, 32), (32, 64), (64, 128), (128, 256), (256, 513))


def measure_loop(index, gpu_index, k: int = 10, per_bin: int = 24, seed: int = 0):
    """Per-query latency of the C++ matcher against the persistent serving kernel
    (``GpuRuleIndex.query_loop``: one request, one round trip) by merged-row size: returns (the
    smallest merged size from which the loop answers every larger bin at least as fast, or None;
    {bin: (cpu_us, loop_us, queries)}).  The native front then sends a query to the loop when
    its merged rows reach that size (SERVE_BACKEND=auto)."""
    import numpy as np
    keys = np.nonzero(index.is_key)[0].astype(np.int32)
    if len(keys) == 0:
        return None, {}
    rp = np.asarray(index.row_ptr)
    rl = rp[keys + 1] - rp[keys]
    rng = np.random.default_rng(seed)
    host = index.native()
    res = {}
    for lo, hi in MERGE_BINS:
        qs = []
        for _ in range(4000):
            n = int(rng.integers(1, 6))
            pick = rng.integers(0, len(keys), n)
            if lo <= int(rl[pick].sum()) < hi:
                qs.append(keys[pick])
            if len(qs) >= per_bin:
                break
        if not qs:
            continue
        tc, tg = [], []
        for q in qs:
            q_ptr = np.array([0, len(q)], np.int64)
            if not gpu_index.query_loop(q_ptr, q, k)[2]:
                return None, {}
            t0 = time.perf_counter()
            host.query_batch(q_ptr, q, k)
            tc.append(time.perf_counter() - t0)
            t0 = time.perf_counter()
            gpu_index.query_loop(q_ptr, q, k)
            tg.append(time.perf_counter() - t0)
        res[f"{lo}-{hi - 1}"] = (round(float(np.median(tc)) * 1e6, 2),
                                 round(float(np.median(tg)) * 1e6, 2), len(qs))
    best = None
    for (lo, hi) in reversed(MERGE_BINS):  # the suffix of bins where the loop is no slower
        r = res.get(f"{lo}-{hi - 1}")
        if r is None:
            continue
        if r[1] <= r[0]:
            best = lo
        else:
            break
    return best, res


class ReloadManager:
    """Owns the current snapshot; thread-safe reload with single-assignment swap."""

    def __init__(self, cfg: ApiSettings, gpu_factory=None):
        self.cfg = cfg
        self.snapshot: Optional[ModelSnapshot] = None
        self.reload_counter = 0
        self.failed_reloads = 0
        self.last_error: Optional[str] = None
        self._lock = threading.Lock()
        self._gpu_factory = gpu_factory
        self.last_reload_seconds = 0.0
        # called with every new snapshot right after the swap (the native front's model push)
        self.listeners: List[Any] = []

    # -- reference-compatible accessors -------------------------------------------------
    @property
    def finished_loading(self) -> bool:
        return self.snapshot is not None

    @property
    def cache_value(self) -> Optional[str]:
        s = self.snapshot
        return s.marker if s is not None else None

    def read_marker(self) -> Optional[str]:
        p = self.cfg.cache_file
        if not p.exists():
            return None
        with open(p, "r") as f:
            return f.read()

    def is_data_stale(self) -> bool:
        marker = self.read_marker()
        if marker is None:
            logger.info("Cache file does not exist")
            return True
        current = self.cache_value
        if current != marker:
            logger.info(f"Data is stale, current value is {current} and last value was {marker}")
            return True
        return False

    def reload_data_if_required(self) -> bool:
        with self._lock:
            if not self.is_data_stale() and self.finished_loading:
                logger.info("data is not stale, no need to reload")
                return False
            return self._perform_reload()

    def _perform_reload(self) -> bool:
        logger.info("Reloading data!")
        t0 = time.perf_counter()
        marker = self.read_marker()
        try:
            best, index, source = read_pickle_dict(self.cfg)
            gpu_index = self._gpu_factory(index) if self._gpu_factory else None
            gmb, cross, gmm, lcross = None, None, None, None
            if gpu_index is not None:
                if self.cfg.serve_backend == "hip":  # forced: every batch on the GPU
                    gmb = 1
                elif self.cfg.serve_backend == "loop":  # forced: the serving kernel
                    gmm = 0
                else:
                    gmb, cross = measure_crossover(index, gpu_index)
                    if hasattr(gpu_index, "query_loop"):  # the serving kernel is optional
                        try:
                            gmm, lcross = measure_loop(index, gpu_index)
                        except Exception as e:  # the loop stays off; batches still measured
                            logger.warning(f"serving-loop measurement failed ({e}); loop off")
        except Exception as e:  # keep serving the previous snapshot; retry next tick
            self.failed_reloads += 1
            self.last_error = f"{type(e).__name__}: {e}"
            logger.error(f"Reload failed ({self.last_error}); keeping the previous model")
            return False
        # the marker may have moved while we were reading: re-read, and only commit the value
        # we read BEFORE loading (a later change triggers another reload next tick)
        snap = ModelSnapshot(best, index, marker, time.time(), index.n_keys, source, gpu_index,
                             gmb, cross, gmm, lcross)
        if gpu_index is not None:
            logger.info(f"HIP matcher crossover: batches >= {gmb} go to the GPU" if gmb else
                        "HIP matcher never beats the C++ matcher on this index: CPU only")
            if gmm is not None:
                logger.info(f"HIP serving loop: queries merging >= {gmm} entries go to the GPU")
        self.snapshot = snap  # single reference assignment = atomic swap
        for fn in list(self.listeners):
            try:
                fn(snap)
            except Exception as e:  # a listener must not undo a good reload
                logger.error(f"snapshot listener failed: {e!r}")
        self.reload_counter += 1
        self.last_error = None
        self.last_reload_seconds = time.perf_counter() - t0
        logger.info("Finished reloading, should reflect changes. "
                    f"Data was reloaded {self.reload_counter} times")
        return True
