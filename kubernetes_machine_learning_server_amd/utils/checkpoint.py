"""Phase-level checkpoint / resume for the job (SURVEY §5.4 "New").

The reference job is idempotent per run and restarts from scratch (``machine-learning/main.py``
has no intra-run state; K8s ``restartPolicy: OnFailure`` re-runs it, ``job.yaml:41``).  That is
fine for a 1-minute CPU job but not for a 100M-transaction multi-GPU run, so expensive phases
persist their outputs under ``KMLS_CHECKPOINT_DIR`` keyed by (dataset path, size, mtime,
min_support, rules mode, sample ratio).  A crashed job that restarts on the same dataset (the
rotation cursor only advances after success) resumes at the first missing phase; a successful
run deletes its checkpoint.  Files are ``.npz`` written atomically and read with
``allow_pickle=False`` — nothing in a checkpoint can execute code.
"""
from __future__ import annotations

import hashlib
import io
import json
import os
import pathlib
import shutil
from typing import Dict, Optional

import numpy as np

from .atomic_io import atomic_write_bytes


class PhaseCheckpoint:
    def __init__(self, root: Optional[os.PathLike], key: Dict):
        self.enabled = root is not None
        digest = hashlib.sha256(json.dumps(key, sort_keys=True, default=str).encode()).hexdigest()
        self.dir = pathlib.Path(root) / digest[:20] if root is not None else None
        self.key = key

    @classmethod
    def for_dataset(cls, root: Optional[os.PathLike], dataset: str, **params) -> "PhaseCheckpoint":
        st = os.stat(dataset)
        key = {"dataset": os.path.abspath(dataset), "size": st.st_size, "mtime_ns": st.st_mtime_ns}
        key.update(params)
        return cls(root, key)

    def _path(self, phase: str) -> pathlib.Path:
        return self.dir / f"{phase}.npz"

    def has(self, phase: str) -> bool:
        return self.enabled and self._path(phase).exists()

    def save(self, phase: str, **arrays) -> None:
        if not self.enabled:
            return
        buf = io.BytesIO()
        np.savez(buf, **{k: np.asarray(v) for k, v in arrays.items()})
        atomic_write_bytes(self._path(phase), buf.getvalue())
        atomic_write_bytes(self.dir / "key.json", json.dumps(self.key, default=str).encode())

    def load(self, phase: str) -> Optional[Dict[str, np.ndarray]]:
        if not self.has(phase):
            return None
        with np.load(self._path(phase), allow_pickle=False) as z:
            return {k: z[k] for k in z.files}

    def clear(self) -> None:
        if self.enabled and self.dir.exists():
            shutil.rmtree(self.dir, ignore_errors=True)
