"""Synthetic Prometheus-like series generators.

* ``seasonal`` — level + daily seasonality + trend + noise (deterministic in
  the timestamp, so any window can be re-queried consistently);
* ``error_rate`` — low 5xx rate (~0.1-0.7/s) like the reference demo's
  normal replay, with optional spikes (~40/s) like its fault replay
  (``examples/spring-boot-demo/src/main/resources/data{1,2}.txt``); the
  values here are generated, not copied;
* ``step_change`` — multiply a base generator after a switch time
  (a regressed canary).
"""

from __future__ import annotations

from typing import Callable, Optional, Sequence

import numpy as np

Gen = Callable[[np.ndarray], np.ndarray]


def _hash_noise(ts: np.ndarray, seed: int) -> np.ndarray:
    """Deterministic N(0,1)-ish noise from the timestamp (stable re-queries)."""
    x = (np.asarray(ts, dtype=np.int64) // 1) * 2654435761 + seed * 40503
    x = (x ^ (x >> 13)) * 1274126177
    x = x ^ (x >> 16)
    u1 = ((x & 0xFFFF) + 1) / 65537.0
    u2 = (((x >> 16) & 0xFFFF) + 1) / 65537.0
    return np.sqrt(-2 * np.log(u1)) * np.cos(2 * np.pi * u2)


def seasonal(level: float = 50.0, amp: float = 10.0, period: float = 86400.0, noise: float = 1.0,
             trend: float = 0.0, seed: int = 0, phase: float = 0.0, t0: float = 0.0) -> Gen:
    """``trend`` is in units per hour relative to ``t0``."""
    def f(ts):
        ts = np.asarray(ts, dtype=np.float64)
        return (level + trend * (ts - t0) / 3600.0
                + amp * np.sin(2 * np.pi * ts / period + phase) + noise * _hash_noise(ts, seed))
    return f


def error_rate(base: float = 0.3, spread: float = 0.2, seed: int = 0,
               spikes: Optional[Sequence[float]] = None, spike_value: float = 40.0) -> Gen:
    """Low error rate around ``base``; ``spikes`` are absolute timestamps (s)
    at which the rate jumps to ``spike_value``."""
    spikes = np.asarray(spikes if spikes is not None else [], dtype=np.float64)

    def f(ts):
        ts = np.asarray(ts, dtype=np.float64)
        v = np.clip(base + spread * 0.5 * _hash_noise(ts, seed), 0.0, None)
        if spikes.size:
            hit = np.isin(np.round(ts / 60.0), np.round(spikes / 60.0))
            v = np.where(hit, spike_value + 0.5 * _hash_noise(ts, seed + 1), v)
        return v
    return f


def step_change(base: Gen, at: float, factor: float = 3.0, add: float = 0.0) -> Gen:
    def f(ts):
        ts = np.asarray(ts, dtype=np.float64)
        v = base(ts)
        return np.where(ts >= at, v * factor + add, v)
    return f


def gaps(base: Gen, every: int = 17) -> Gen:
    def f(ts):
        v = np.asarray(base(ts), dtype=np.float64).copy()
        idx = (np.asarray(ts, dtype=np.int64) // 60) % every == 0
        v[idx] = np.nan
        return v
    return f


def replay(rates: Sequence[float], start: float, step: float = 60.0, before: Optional[Gen] = None,
           loop: bool = False) -> Gen:
    """Replay a recorded rate file (one value per ``step`` from ``start``), like
    the reference demo's ``FileErrorGenerator``; before ``start`` the ``before``
    generator (history), after the end NaN (or wrap around with ``loop``)."""
    r = np.asarray(rates, dtype=np.float64)

    def f(ts):
        ts = np.asarray(ts, dtype=np.float64)
        k = np.floor((ts - start) / step).astype(np.int64)
        if loop:
            k = np.where(k >= 0, k % len(r), k)
        inside = (k >= 0) & (k < len(r))
        out = np.full(ts.shape, np.nan)
        out[inside] = r[k[inside]]
        if before is not None:
            out = np.where(k < 0, before(ts), out)
        return out
    return f


def read_rates(path: str) -> list:
    with open(path) as fh:
        return [float(x) for x in (ln.strip() for ln in fh) if x and not x.startswith("#")]
