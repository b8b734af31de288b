"""Crash-safe artifact writes for the PVC file protocol.

The reference writes pickles in place (``machine-learning/main.py:144-145``) so a reader that
polls during a write can load a truncated file.  Here every artifact is written to a temp file
in the same directory, fsync'ed, then ``os.replace``d over the target (atomic on POSIX), and
the directory is fsync'ed.  The marker file is still written LAST, so readers reload only
after every artifact of a run is complete.
"""
from __future__ import annotations

import os
import pathlib
import pickle
import tempfile
from typing import Any, Union

PathLike = Union[str, os.PathLike]


def _fsync_dir(d: pathlib.Path) -> None:
    try:
        fd = os.open(str(d), os.O_RDONLY)
    except OSError:
        return
    try:
        os.fsync(fd)
    except OSError:
        pass
    finally:
        os.close(fd)


def atomic_write_bytes(path: PathLike, data: bytes, mode: int = 0o644) -> None:
    """Write-to-temp + fsync + rename.  ``mode`` is applied before the rename (mkstemp creates
    0600 files, which other pods' UIDs could not read on a shared RWX volume)."""
    p = pathlib.Path(path)
    p.parent.mkdir(parents=True, exist_ok=True)
    fd, tmp = tempfile.mkstemp(prefix=f".{p.name}.", suffix=".tmp", dir=str(p.parent))
    try:
        with os.fdopen(fd, "wb") as f:
            f.write(data)
            f.flush()
            os.fsync(f.fileno())
        os.chmod(tmp, mode)
        os.replace(tmp, p)
    except BaseException:
        try:
            os.unlink(tmp)
        except OSError:
            pass
        raise
    _fsync_dir(p.parent)


def atomic_write_with(path: PathLike, write, mode: int = 0o644) -> None:
    """``atomic_write_bytes`` for large artifacts: ``write(file)`` streams into the temp file
    (no in-memory copy of the whole artifact), then fsync + rename as above."""
    p = pathlib.Path(path)
    p.parent.mkdir(parents=True, exist_ok=True)
    fd, tmp = tempfile.mkstemp(prefix=f".{p.name}.", suffix=".tmp", dir=str(p.parent))
    try:
        with os.fdopen(fd, "wb") as f:
            write(f)
            f.flush()
            os.fsync(f.fileno())
        os.chmod(tmp, mode)
        os.replace(tmp, p)
    except BaseException:
        try:
            os.unlink(tmp)
        except OSError:
            pass
        raise
    _fsync_dir(p.parent)


def atomic_write_text(path: PathLike, text: str, encoding: str = "utf-8") -> None:
    atomic_write_bytes(path, text.encode(encoding))


def atomic_pickle(path: PathLike, obj: Any) -> None:
    atomic_write_bytes(path, pickle.dumps(obj, protocol=pickle.HIGHEST_PROTOCOL))


def append_line(path: PathLike, line: str, header: str = "") -> None:
    """Append one line (with optional header on creation), fsync'ed."""
    p = pathlib.Path(path)
    p.parent.mkdir(parents=True, exist_ok=True)
    existed = p.exists()
    with open(p, "a", encoding="utf-8") as f:
        if not existed and header:
            f.write(header)
        f.write(line)
        f.flush()
        os.fsync(f.fileno())
