"""Phase timer: wall-clock phases of a job/bench run, emitted as JSON.

With ``KMLS_ROCTX=1`` every phase is also a roctx range (through the native module's roctx
wrapper, ``csrc/host/trace.cpp``), so ``rocprofv3 --marker-trace`` shows the job's phases over
the kernels alongside the native ``kmls.*`` ranges."""
from __future__ import annotations

import contextlib
import json
import os
import time
from typing import Dict, Iterator, List, Optional, Tuple

_ROCTX = None  # native module when roctx ranges are on, False when off


def _roctx():
    global _ROCTX
    if _ROCTX is None:
        _ROCTX = False
        if os.environ.get("KMLS_ROCTX") == "1":
            try:
                from ..ops import native
                m = native.load(build_if_missing=False)
                if m.roctx_enabled():
                    _ROCTX = m
            except Exception:  # pragma: no cover - tracing is best-effort
                _ROCTX = False
    return _ROCTX


class PhaseTimer:
    def __init__(self) -> None:
        self.phases: List[Tuple[str, float]] = []
        self._t0 = time.perf_counter()

    @contextlib.contextmanager
    def phase(self, name: str) -> Iterator[None]:
        rx = _roctx()
        if rx:
            rx.roctx_push(f"kmls.job.{name}")
        t = time.perf_counter()
        try:
            yield
        finally:
            self.phases.append((name, time.perf_counter() - t))
            if rx:
                rx.roctx_pop()

    def add(self, name: str, seconds: float) -> None:
        self.phases.append((name, seconds))

    def as_dict(self) -> Dict[str, float]:
        out: Dict[str, float] = {}
        for k, v in self.phases:
            out[k] = out.get(k, 0.0) + v
        out["total"] = time.perf_counter() - self._t0
        return out

    def to_json(self) -> str:
        return json.dumps({k: round(v, 6) for k, v in self.as_dict().items()})
