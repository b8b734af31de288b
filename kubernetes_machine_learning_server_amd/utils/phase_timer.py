"""Phase timer: wall-clock phases of a job/bench run, emitted as JSON."""
from __future__ import annotations

import contextlib
import json
import time
from typing import Dict, Iterator, List, Tuple


class PhaseTimer:
    def __init__(self) -> None:
        self.phases: List[Tuple[str, float]] = []
        self._t0 = time.perf_counter()

    @contextlib.contextmanager
    def phase(self, name: str) -> Iterator[None]:
        t = time.perf_counter()
        try:
            yield
        finally:
            self.phases.append((name, time.perf_counter() - t))

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
