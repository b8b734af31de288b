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


def _bind_torch_runtime() -> None:
    """Import torch (if installed) BEFORE the extension.

    The ROCm torch wheel ships its own ``libamdhip64.so`` with the same SONAME
    (``libamdhip64.so.7``) as /opt/rocm's.  Loading torch first makes the extension's
    ``NEEDED libamdhip64.so.7`` resolve to the already-loaded runtime, so the process has ONE
    HIP runtime and torch tensors / RCCL collectives and our kernels share devices and streams.
    Loading ours first would leave torch with a second runtime that sees no GPU.
    """
    if os.environ.get("KMLS_NO_TORCH"):
        return
    try:
        import torch  # noqa: F401
    except Exception:
        pass


def load(build_if_missing: bool = True) -> ModuleType:
    global _mod
    if _mod is not None:
        return _mod
    with _lock:
        if _mod is not None:
            return _mod
        _bind_torch_runtime()
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
