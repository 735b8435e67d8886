"""HBM-resident ring buffers for streamed Prometheus range-vectors.

``HistoryRing``: ``[N, R]`` (bf16 by default) — the 7-day history of each
series at the 60 s step (R = 10,080; ``metricsquery.go:43,75``).  100k series
x 10,080 x 2 B = 2 GB per metric type: the whole node's history for every
metric type fits comfortably in one MI355X's 288 GB, so it stays resident and
is never re-fetched; each tick appends one column.

``WindowRing``: ``[N, P*W]`` float32 — the current (canary) window, P pods x
W slots (slot = tick mod W), plus a static baseline window of the same shape.

Logical order of the history: oldest sample at column ``head``, ``length``
valid samples.  Kernels resolve the rotation while staging into LDS, so no
data is ever moved to "un-rotate" the ring.
"""

from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch


@dataclass
class RingState:
    head: int = 0
    length: int = 0


class HistoryRing:
    def __init__(self, n: int, ring_len: int, dtype=torch.bfloat16, device="cpu") -> None:
        self.n = n
        self.R = ring_len
        # pad rows to a multiple of 16 bytes so vector loads stay aligned
        elt = torch.tensor([], dtype=dtype).element_size()
        per16 = 16 // elt
        self.ld = ((ring_len + per16 - 1) // per16) * per16
        self._store = torch.full((n, self.ld), float("nan"), dtype=dtype, device=device)
        self.data = self._store[:, :ring_len]
        self.state = RingState()

    @property
    def head(self) -> int:
        return self.state.head

    @property
    def length(self) -> int:
        return self.state.length

    def load(self, values: torch.Tensor) -> None:
        """Fill from a logical ``[N, T]`` block (T <= R); oldest first."""
        T = values.shape[1]
        if T > self.R:
            values = values[:, -self.R:]
            T = self.R
        self.data[:, :T].copy_(values.to(self.data.dtype))
        self.state = RingState(head=0, length=T)

    def next_col(self) -> int:
        return (self.state.head + self.state.length) % self.R

    def advance(self, k: int = 1) -> None:
        for _ in range(k):
            if self.state.length < self.R:
                self.state.length += 1
            else:
                self.state.head = (self.state.head + 1) % self.R

    def append_(self, values: torch.Tensor) -> None:
        """Host-driven append of ``[N, S]`` (reference path; the GPU path uses
        ``ops.kernels.ring_append`` / ``tick_ingest``)."""
        S = values.shape[1]
        for j in range(S):
            self.data[:, self.next_col()] = values[:, j].to(self.data.dtype)
            self.advance(1)

    def logical(self) -> torch.Tensor:
        """``[N, length]`` in time order (copies; for tests and CPU paths)."""
        idx = (torch.arange(self.state.length, device=self.data.device) + self.state.head) % self.R
        return self.data.index_select(1, idx)


class WindowRing:
    """Current window: P pods x W slots; slot = tick mod W."""

    def __init__(self, n: int, pods: int, window: int, device="cpu") -> None:
        self.n, self.P, self.W = n, pods, window
        self.data = torch.full((n, pods * window), float("nan"), dtype=torch.float32, device=device)
        self.ticks = 0

    def slot(self) -> int:
        return self.ticks % self.W

    def horizons(self, ticks_done: int | None = None) -> np.ndarray:
        """Forecast horizon (steps after the history end) of every column after
        ``ticks_done`` ticks have been ingested (newest slot = (ticks-1) mod W)."""
        k = (self.ticks if ticks_done is None else ticks_done) - 1
        W = self.W
        if k < 0:
            h = np.arange(1, W + 1)
        else:
            newest = k % W
            hn = min(k + 1, W)
            age = (newest - np.arange(W)) % W
            h = hn - age
            h = np.where(h >= 1, h, W + h)  # unwritten slots (NaN) keep a valid horizon
        return np.tile(h.astype(np.int32), self.P)

    def push_(self, values: torch.Tensor) -> torch.Tensor:
        """Reference (host-driven) tick: returns the pod-mean of the evicted slot."""
        s = self.slot()
        cols = torch.arange(self.P, device=self.data.device) * self.W + s
        old = self.data[:, cols].clone()
        self.data[:, cols] = values.float()
        self.ticks += 1
        valid = ~torch.isnan(old)
        cnt = valid.sum(1)
        mean = torch.where(valid, old, torch.zeros_like(old)).sum(1) / cnt.clamp(min=1)
        return torch.where(cnt > 0, mean, torch.full_like(mean, float("nan")))
