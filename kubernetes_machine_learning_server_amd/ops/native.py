"""Loader for the in-tree native extension (``_native``: C++ runtime + gfx950 HIP kernels).

The extension is built in-tree (``ops/build.py``) so that the same ``.so`` travels to the GPU
box.  If it is missing we try to build it once (hipcc is in the image); if that fails we raise
loudly — there is no silent pure-Python fallback for the GPU path.
"""
from __future__ import annotations

import importlib
import os
import threading
from types import ModuleType

_lock = threading.Lock()
_mod: "ModuleType | None" = None


class NativeUnavailable(RuntimeError):
    pass


def load(build_if_missing: bool = True) -> ModuleType:
    global _mod
    if _mod is not None:
        return _mod
    with _lock:
        if _mod is not None:
            return _mod
        try:
            _mod = importlib.import_module("kubernetes_machine_learning_server_amd._native")
            return _mod
        except ImportError as first:
            if not build_if_missing or os.environ.get("KMLS_NO_AUTOBUILD"):
                raise NativeUnavailable(f"kmls native extension not built: {first}") from first
        from . import build as _build
        try:
            _build.build()
        except Exception as e:  # pragma: no cover - toolchain failure
            raise NativeUnavailable(f"kmls native extension missing and build failed: {e}") from e
        importlib.invalidate_caches()
        _mod = importlib.import_module("kubernetes_machine_learning_server_amd._native")
        return _mod


def gpu_available() -> bool:
    """True iff a HIP device is visible (does not initialise torch)."""
    if os.environ.get("KMLS_FORCE_CPU"):
        return False
    try:
        return bool(load().gpu_available())
    except NativeUnavailable:
        return False


def require_gpu() -> ModuleType:
    m = load()
    if not m.gpu_available():
        raise NativeUnavailable("no HIP device visible: the GPU path cannot run here")
    return m


def so_path() -> str:
    return load().__file__
