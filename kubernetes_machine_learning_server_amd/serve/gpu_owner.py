"""One GPU-owning matcher process shared by all uvicorn workers.

The reference runs a single worker (``rest_api/Dockerfile:28``). Here ``--workers N`` gives N
processes. Without an owner, every worker would build its own HBM index and launch its own small
batches. With an owner, only ONE process opens the GPU:

* **Owner (``GpuOwner``).** It runs its own ``ReloadManager`` on the same volume and marker, so
  it hot-reloads the same ``rules.idx``. It keeps one ``GpuRuleIndex`` and serves batches from
  every worker. Each worker holds a shared-memory segment. The owner's selector loop collects
  the batches that are ready across workers, answers them with ONE kernel launch, and writes
  each worker's results back into that worker's segment.
* **Worker (``OwnerClient``).** It stands in for ``GpuRuleIndex`` in the worker's snapshot, with
  the same ``query_batch(q_ptr, seeds, k)``. It copies the queries into its segment and sends a
  16-byte doorbell over a Unix socket. It then waits for the owner's doorbell and reads the
  results from the segment. The crossover measured at index load (``state.measure_crossover``)
  therefore covers the whole IPC + kernel path.

Consistency: each request carries the fingerprint of the worker's index
(``index.index_fingerprint``). The owner answers only when its loaded index has the same
fingerprint. Otherwise it returns -2 for every query, and the worker's micro-batcher answers
them with the C++ matcher. During a reload no query is ever answered from a different model.
"""
from __future__ import annotations

import logging
import os
import selectors
import socket
import struct
import threading
import time
from multiprocessing import shared_memory
from typing import Callable, Dict, Optional

import numpy as np

logger = logging.getLogger("kmls.api")

_HELLO = struct.Struct("<I64s")      # magic, shared-memory segment name
_REQ = struct.Struct("<QiiqI")       # fingerprint, k, B, ns, seq
_RESP = struct.Struct("<iI")         # status (0 ok, 1 stale model, 2 error), seq
_MAGIC = 0x4B4D4C53                  # "KMLS"
SEG_BYTES = int(os.environ.get("KMLS_OWNER_SEG_MB", "16")) << 20


def _recv_exact(sock: socket.socket, n: int) -> bytes:
    buf = bytearray()
    while len(buf) < n:
        chunk = sock.recv(n - len(buf))
        if not chunk:
            raise ConnectionError("GPU owner connection closed")
        buf += chunk
    return bytes(buf)


def _layout(B: int, ns: int, k: int):
    """Offsets in a worker segment: q_ptr int64[B+1] | seeds int32[ns] | ids int32[B*k] | n int32[B]."""
    o_q = 0
    o_s = o_q + 8 * (B + 1)
    o_i = (o_s + 4 * ns + 7) & ~7
    o_n = o_i + 4 * B * k
    end = o_n + 4 * B
    return o_q, o_s, o_i, o_n, end


class OwnerClient:
    """Worker side: looks like a GpuRuleIndex bound to one index fingerprint."""

    def __init__(self, path: str, fingerprint: int, timeout_s: float = 5.0):
        self.path = path
        self.fingerprint = int(fingerprint) & 0xFFFFFFFFFFFFFFFF
        self.timeout_s = timeout_s
        self._lock = threading.Lock()
        self._sock: Optional[socket.socket] = None
        self._shm: Optional[shared_memory.SharedMemory] = None
        self._seq = 0
        self.calls = 0
        self.stale = 0

    def _connect(self):
        if self._sock is not None:
            return
        shm = shared_memory.SharedMemory(create=True, size=SEG_BYTES)
        s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        s.settimeout(self.timeout_s)
        try:
            s.connect(self.path)
            s.sendall(_HELLO.pack(_MAGIC, shm.name.encode()))
        except Exception:
            s.close()
            shm.close()
            shm.unlink()
            raise
        self._sock, self._shm = s, shm

    def close(self):
        with self._lock:
            if self._sock is not None:
                self._sock.close()
                self._sock = None
            if self._shm is not None:
                self._shm.close()
                try:
                    self._shm.unlink()
                except FileNotFoundError:
                    pass
                self._shm = None

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass

    def wait_ready(self, timeout_s: float = 10.0) -> bool:
        """Until the owner has loaded this model (empty probes); False on timeout."""
        deadline = time.monotonic() + timeout_s
        while time.monotonic() < deadline:
            _, n = self.query_batch(np.zeros(1, np.int64), np.zeros(0, np.int32), 1, probe=True)
            if n is not None:
                return True
            time.sleep(0.05)
        return False

    def query_batch(self, q_ptr, seeds, k: int, probe: bool = False):
        q_ptr = np.ascontiguousarray(q_ptr, np.int64)
        seeds = np.ascontiguousarray(seeds, np.int32)
        B = len(q_ptr) - 1
        ns = int(q_ptr[-1] - q_ptr[0])
        o_q, o_s, o_i, o_n, end = _layout(B, ns, k)
        stale = (np.full((B, k), -1, np.int32), np.full(B, -2, np.int32))
        if end > SEG_BYTES:  # too big for the segment: the caller's CPU path answers
            return stale
        with self._lock:
            try:
                self._connect()
                buf = self._shm.buf
                np.frombuffer(buf, np.int64, B + 1, o_q)[:] = q_ptr - q_ptr[0]
                np.frombuffer(buf, np.int32, ns, o_s)[:] = seeds[q_ptr[0]:q_ptr[-1]]
                self._seq = (self._seq + 1) & 0xFFFFFFFF
                self._sock.sendall(_REQ.pack(self.fingerprint, k, B, ns, self._seq))
                status, seq = _RESP.unpack(_recv_exact(self._sock, _RESP.size))
                if seq != self._seq:
                    raise ConnectionError("GPU owner reply out of sequence")
                self.calls += 1
                if status != 0:
                    self.stale += 1
                    return (None, None) if probe else stale
                if probe:
                    return None, np.zeros(0, np.int32)
                ids = np.frombuffer(buf, np.int32, B * k, o_i).reshape(B, k).copy()
                n = np.frombuffer(buf, np.int32, B, o_n).copy()
                return ids, n
            except (OSError, ConnectionError) as e:
                logger.error(f"GPU owner unavailable ({e!r}); answering on the CPU")
                if self._sock is not None:
                    self._sock.close()
                    self._sock = None
                if self._shm is not None:
                    self._shm.close()
                    try:
                        self._shm.unlink()
                    except FileNotFoundError:
                        pass
                    self._shm = None
                return (None, None) if probe else stale


class _Conn:
    def __init__(self, sock: socket.socket, shm: shared_memory.SharedMemory):
        self.sock = sock
        self.shm = shm
        self.pending = None  # (fingerprint, k, B, ns, seq)


class GpuOwner:
    """Owner side.  ``index_source()`` returns (fingerprint, gpu_index) of the loaded model, or
    (None, None); ``serve_forever`` runs the selector loop until ``stop()``."""

    def __init__(self, path: str, index_source: Callable[[], tuple]):
        self.path = path
        self.index_source = index_source
        self.batches = 0
        self.queries = 0
        self.max_fused = 0
        self._stop = threading.Event()
        self._sel = selectors.DefaultSelector()
        self._conns: Dict[int, _Conn] = {}
        if os.path.exists(path):
            os.unlink(path)
        self._lsock = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        self._lsock.bind(path)
        self._lsock.listen(128)
        self._lsock.setblocking(False)
        self._sel.register(self._lsock, selectors.EVENT_READ, None)

    def stop(self):
        self._stop.set()

    def _accept(self):
        s, _ = self._lsock.accept()
        s.setblocking(True)
        s.settimeout(5.0)
        try:
            magic, name = _HELLO.unpack(_recv_exact(s, _HELLO.size))
            if magic != _MAGIC:
                raise ConnectionError("bad hello")
            shm = shared_memory.SharedMemory(name=name.rstrip(b"\0").decode())
            try:  # the worker owns the segment: keep this process's tracker from unlinking it
                from multiprocessing import resource_tracker
                resource_tracker.unregister(shm._name, "shared_memory")
            except Exception:
                pass
        except Exception as e:
            logger.error(f"GPU owner: rejected a worker ({e!r})")
            s.close()
            return
        s.setblocking(False)
        self._conns[s.fileno()] = _Conn(s, shm)
        self._sel.register(s, selectors.EVENT_READ, s.fileno())

    def _drop(self, fd: int):
        c = self._conns.pop(fd, None)
        if c is None:
            return
        try:
            self._sel.unregister(c.sock)
        except Exception:
            pass
        c.sock.close()
        c.shm.close()  # the worker owns (and unlinks) its segment

    def _read_request(self, fd: int) -> None:
        c = self._conns[fd]
        try:
            c.sock.setblocking(True)
            c.sock.settimeout(5.0)
            c.pending = _REQ.unpack(_recv_exact(c.sock, _REQ.size))
        except (OSError, ConnectionError):
            self._drop(fd)
        finally:
            if fd in self._conns:
                c.sock.setblocking(False)

    def _answer(self) -> None:
        """One fused launch for every pending request whose model matches the loaded one."""
        ready = [c for c in self._conns.values() if c.pending is not None]
        if not ready:
            return
        fp, gidx = self.index_source()
        by_k: Dict[int, list] = {}
        for c in ready:
            f, k, B, ns, seq = c.pending
            if gidx is None or f != fp:
                self._reply(c, 1, seq)
            else:
                by_k.setdefault(k, []).append(c)
        for k, conns in by_k.items():
            if all(c.pending[2] == 0 for c in conns):  # readiness probes (no queries)
                for c in conns:
                    self._reply(c, 0, c.pending[4])
                continue
            qs, ss, sizes = [], [], []
            base = 0
            for c in conns:
                _, _, B, ns, _ = c.pending
                o_q, o_s, o_i, o_n, _ = _layout(B, ns, k)
                q = np.frombuffer(c.shm.buf, np.int64, B + 1, o_q)
                qs.append(q[:-1] + base)
                ss.append(np.frombuffer(c.shm.buf, np.int32, ns, o_s))
                sizes.append(B)
                base += ns
            q_all = np.concatenate(qs + [np.array([base], np.int64)])
            s_all = np.concatenate(ss) if ss else np.zeros(0, np.int32)
            try:
                ids, n = gidx.query_batch(q_all, s_all, k)
                status = 0
            except Exception as e:  # pragma: no cover - surfaced as a stale reply
                logger.error(f"GPU owner: batch failed ({e!r})")
                status = 2
            self.batches += 1
            self.queries += int(sum(sizes))
            self.max_fused = max(self.max_fused, len(conns))
            row = 0
            for c, B in zip(conns, sizes):
                _, _, _, ns, seq = c.pending
                if status == 0:
                    o_q, o_s, o_i, o_n, _ = _layout(B, ns, k)
                    np.frombuffer(c.shm.buf, np.int32, B * k, o_i)[:] = ids[row:row + B].ravel()
                    np.frombuffer(c.shm.buf, np.int32, B, o_n)[:] = n[row:row + B]
                row += B
                self._reply(c, status, seq)

    def _reply(self, c: _Conn, status: int, seq: int) -> None:
        c.pending = None
        try:
            c.sock.setblocking(True)
            c.sock.sendall(_RESP.pack(status, seq))
            c.sock.setblocking(False)
        except OSError:
            self._drop(c.sock.fileno())

    def serve_forever(self, poll_s: float = 0.05) -> None:
        try:
            while not self._stop.is_set():
                events = self._sel.select(timeout=poll_s)
                for key, _ in events:
                    if key.data is None:
                        self._accept()
                    else:
                        self._read_request(key.data)
                # requests that became ready while the first was read join the same launch
                for key, _ in self._sel.select(timeout=0):
                    if key.data is not None and self._conns.get(key.data) is not None \
                            and self._conns[key.data].pending is None:
                        self._read_request(key.data)
                self._answer()
        finally:
            for fd in list(self._conns):
                self._drop(fd)
            self._sel.close()
            self._lsock.close()
            if os.path.exists(self.path):
                os.unlink(self.path)


def owner_main(path: str) -> int:  # pragma: no cover - process entry (GPU box)
    """Owner process entry: hot-reloading model + HBM index + selector loop."""
    from ..config import ApiSettings
    from .app import _gpu_factory, _setup_logging
    from .index import index_fingerprint
    from .state import ReloadManager

    _setup_logging()
    cfg = ApiSettings.from_env()
    factory = _gpu_factory(cfg, allow_owner=False)
    if factory is None:  # no HIP device: no socket, the workers stay on the CPU matcher
        logger.info("GPU owner: no HIP device visible, exiting")
        return 0
    mgr = ReloadManager(cfg, gpu_factory=factory)
    fps: Dict[int, int] = {}

    def source():
        snap = mgr.snapshot
        if snap is None or snap.gpu_index is None:
            return None, None
        fp = fps.get(id(snap))
        if fp is None:
            fps.clear()
            fp = fps[id(snap)] = index_fingerprint(snap.index)
        return fp, snap.gpu_index

    owner = GpuOwner(path, source)
    period = max(1.0, 60.0 * cfg.polling_wait_in_minutes)

    def poll():
        while not owner._stop.is_set():
            try:
                mgr.reload_data_if_required()
            except Exception as e:
                logger.error(f"GPU owner reload failed: {e}")
            owner._stop.wait(period)
    threading.Thread(target=poll, daemon=True).start()
    logger.info(f"GPU owner serving on {path}")
    owner.serve_forever()
    return 0
