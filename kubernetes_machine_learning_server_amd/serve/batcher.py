"""Async request micro-batcher feeding the HIP matcher (SURVEY §2.E "intra-process concurrency").

Requests already queued when the batcher wakes are concatenated into one CSR query batch; one
``serve_match_topk`` launch answers all of them (one workgroup per query) and the futures are
resolved on the event loop.  The batcher only WAITS (up to ``BATCH_WAIT_US``, until
``BATCH_MAX``) when recent load shows that waiting fills a GPU-sized batch — at low QPS a
timer would only add latency.  Batches smaller than ``GPU_MIN_BATCH`` are answered inline by
the C++ CPU matcher (~1 µs/query; an executor hop alone costs ~50 µs); GPU batches run in a
worker thread (the native call releases the GIL), so the event loop keeps accepting requests
while a batch is in flight.
"""
from __future__ import annotations

import asyncio
import time
from typing import List, Optional, Tuple

import numpy as np


class MicroBatcher:
    def __init__(self, max_batch: int = 256, max_wait_us: int = 200, gpu_min_batch: int = 16):
        self.max_batch = max(1, int(max_batch))
        self.max_wait = max(0, int(max_wait_us)) / 1e6
        self.gpu_min_batch = int(gpu_min_batch)
        self._q: Optional[asyncio.Queue] = None
        self._task: Optional[asyncio.Task] = None
        self.batches = 0
        self.gpu_batches = 0
        self.queries = 0
        self.last_batch = 0
        self._load = 0.0  # EWMA of the immediately-available batch size

    def start(self) -> None:
        if self._task is None:
            self._q = asyncio.Queue()
            self._task = asyncio.get_running_loop().create_task(self._run())

    async def stop(self) -> None:
        if self._task is not None:
            self._task.cancel()
            try:
                await self._task
            except (asyncio.CancelledError, Exception):
                pass
            self._task = None

    async def submit(self, snap, ids: np.ndarray, k: int) -> Tuple[np.ndarray, int]:
        """Returns (ids[k], n) for one query; n == -1 → no seed is a key."""
        fut = asyncio.get_running_loop().create_future()
        await self._q.put((snap, ids, k, fut))
        return await fut

    async def _run(self) -> None:
        loop = asyncio.get_running_loop()
        while True:
            first = await self._q.get()
            items = [first]
            while len(items) < self.max_batch:  # drain what is already queued
                try:
                    items.append(self._q.get_nowait())
                except asyncio.QueueEmpty:
                    break
            self._load = 0.8 * self._load + 0.2 * len(items)
            gmin = self._gpu_min(first[0])
            if (gmin is not None and self.max_wait > 0 and len(items) < gmin
                    and self._load * 4 >= gmin):
                deadline = time.perf_counter() + self.max_wait
                while len(items) < self.max_batch:
                    rem = deadline - time.perf_counter()
                    if rem <= 0:
                        break
                    try:
                        items.append(await asyncio.wait_for(self._q.get(), rem))
                    except asyncio.TimeoutError:
                        break
            # group by (snapshot, k): a reload between requests must not mix indices
            groups = {}
            for it in items:
                groups.setdefault((id(it[0]), it[2]), []).append(it)
            for (_, k), grp in groups.items():
                snap = grp[0][0]
                try:
                    gmin = self._gpu_min(snap)
                    if gmin is not None and len(grp) >= gmin:
                        ids, n = await loop.run_in_executor(None, self._run_batch, snap, grp, k)
                    else:
                        ids, n = self._run_batch(snap, grp, k)
                    for j, it in enumerate(grp):
                        if not it[3].done():
                            it[3].set_result((ids[j], int(n[j])))
                except Exception as e:  # pragma: no cover - surfaced to the requests
                    for it in grp:
                        if not it[3].done():
                            it[3].set_exception(e)

    def _gpu_min(self, snap) -> Optional[int]:
        """Smallest batch routed to the HIP matcher for this snapshot: its measured crossover
        (state.measure_crossover), never below GPU_MIN_BATCH; None = CPU only."""
        if snap.gpu_index is None:
            return None
        m = getattr(snap, "gpu_min_batch", self.gpu_min_batch)
        if m is None:
            return None
        return max(int(m), 1) if m == 1 else max(int(m), self.gpu_min_batch)

    def _run_batch(self, snap, grp: List, k: int):
        lens = [len(it[1]) for it in grp]
        q_ptr = np.zeros(len(grp) + 1, np.int64)
        np.cumsum(lens, out=q_ptr[1:])
        seeds = np.concatenate([it[1] for it in grp]) if grp else np.zeros(0, np.int32)
        self.batches += 1
        self.queries += len(grp)
        self.last_batch = len(grp)
        gmin = self._gpu_min(snap)
        if gmin is not None and len(grp) >= gmin:
            self.gpu_batches += 1
            ids, n = snap.gpu_index.query_batch(q_ptr, seeds.astype(np.int32), k)
            if (n == -2).any():  # kernel table overflow: answer those on the CPU
                cids, cn = snap.index.native().query_batch(q_ptr, seeds.astype(np.int32), k)
                m = n == -2
                ids[m], n[m] = cids[m], cn[m]
            return ids, n
        return snap.index.native().query_batch(q_ptr, seeds.astype(np.int32), k)
