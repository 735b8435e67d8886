"""Parallel, double-buffered decode of a tick's Prometheus responses (K10, host side).

A 100k-series canary tick at one point per pod and minute is ~1M series in
~10 ``query_range`` bodies (one per metric family and canary / baseline pod
set; ~140 MB of JSON).  :class:`TickDecoder` turns them into the ``[rows,
cols]`` float32 block the tick-ingest kernel reads:

* the whole tick is ONE native call
  (:func:`~foremast_amd.ingest.native.decode_tick`): a pool of C++ threads
  NaN-fills the pinned staging block, then decodes every body — split at
  series boundaries into ~4 chunks per thread, so one large body does not
  serialise the tick — scattering each series into its row through an
  open-addressing key index that also learns the response layout (the label
  object that followed each key last tick: a matching byte hash gives the
  next row without parsing the labels); the ctypes call releases the GIL;
* two staging blocks alternate: tick k+1 decodes on the CPU while the GPU
  scores tick k (the caller submits k+1 right after enqueueing tick k's H2D
  copy; block k is reused by tick k+2, after tick k's copy has completed).
"""

from __future__ import annotations

import time
from concurrent.futures import Future, ThreadPoolExecutor
from typing import List, Optional, Sequence

import numpy as np
import torch

from . import native


class TickDecoder:
    def __init__(self, tables: Sequence[native.KeyTable], rows: int, cols: int = 1, pinned: bool = True,
                 threads: int = 8) -> None:
        self.tables = list(tables)
        self.rows, self.cols = rows, cols
        self.bufs = []
        for _ in range(2):
            t = torch.empty((rows, cols), dtype=torch.float32)
            self.bufs.append(t.pin_memory() if pinned else t)
        self.views = [b.numpy() for b in self.bufs]
        self.threads = max(1, threads)
        self.coord = ThreadPoolExecutor(max_workers=1, thread_name_prefix="tick-decode-coord")
        self.i = 0
        self.last_decode_ms = 0.0

    def _decode(self, slot: int, bodies: Sequence[bytes], start: float, step: float):
        out = self.views[slot]
        t0 = time.perf_counter()
        stats = native.decode_tick(bodies, self.tables, start, step, self.cols, out, threads=self.threads)
        self.last_decode_ms = (time.perf_counter() - t0) * 1e3
        return self.bufs[slot], stats

    def submit(self, bodies: Sequence[bytes], start: float, step: float = 60.0) -> Future:
        """Decode one tick's bodies (body j with table j) into the next staging
        block; the future's result is ``(block, [(series, dropped, unmatched)])``
        and ``future.t_submit`` the submit time (detect latency starts there)."""
        if len(bodies) != len(self.tables):
            raise ValueError(f"{len(bodies)} bodies for {len(self.tables)} key tables")
        slot = self.i
        self.i ^= 1
        t_submit = time.perf_counter()
        fut = self.coord.submit(self._decode, slot, bodies, start, step)
        fut.t_submit = t_submit
        return fut

    def close(self) -> None:
        self.coord.shutdown(wait=True)


def pod_matrix_body(metric: str, labels: Sequence[str], ts: float, values: np.ndarray) -> bytes:
    """A ``query_range`` response (one point per series) for pre-rendered label
    objects ``labels[s]`` (e.g. ``'"namespace":"ns","app":"a","pod":"a-c0"'``)."""
    vs = np.char.mod("%.9g", np.asarray(values, dtype=np.float64))  # float32 round-trips exactly
    tsi = int(ts)
    head = '{"metric":{"__name__":"' + metric + '",'
    tail = '"]]}'
    items = [f'{head}{lab}}},"values":[[{tsi},"{v}{tail}' for lab, v in zip(labels, vs.tolist())]
    return ('{"status":"success","data":{"resultType":"matrix","result":[' + ",".join(items) + "]}}").encode()
