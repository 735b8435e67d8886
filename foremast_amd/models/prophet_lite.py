"""Batched Prophet-style additive model (``ML_ALGORITHM=prophet``).

The reference brain lists Prophet among its univariate models
(``docs/guides/design.md:68-72``; ``foremast-brain/README.md:14-20``).  Prophet
fits  y(t) = g(t) + s(t) + e  with a piecewise-linear trend g (changepoints
in the first 80 % of the history, sparse slope changes) and Fourier-series
seasonalities s (daily, weekly), by MAP optimisation per series.

Here the same model family is fit for *all* series of a batch at once as a
weighted ridge regression — one batched ``[B, P, P]`` normal-equation solve
on the GPU (rocBLAS/rocSOLVER via torch) instead of B independent L-BFGS
runs:

* features per series: intercept, scaled time, ``n_changepoints`` hinge
  terms ``max(0, t - c_k)`` (L2-penalised slope changes — the Laplace prior's
  ridge analogue), daily Fourier terms (order 4) when the history spans >= 2
  days, weekly (order 3) when >= 2 weeks — Prophet's auto-enable rules;
* NaN gaps get zero weight;
* the band is ``forecast ± threshold * sigma`` with sigma the residual
  standard deviation (Prophet samples trend uncertainty; the reference
  thresholds the interval the same way, design decision in docs/SCORING.md).
"""

from __future__ import annotations

import math
from dataclasses import dataclass
from typing import List, Tuple

import torch

DAY = 86400.0
WEEK = 7 * DAY


@dataclass
class ProphetFit:
    beta: torch.Tensor        # [B, P]
    sigma: torch.Tensor       # [B]
    n_valid: torch.Tensor     # [B]
    t0: torch.Tensor          # [B] first timestamp
    span: torch.Tensor        # [B] history span (s)
    cps: torch.Tensor         # [B, K] changepoints in scaled time
    yscale: torch.Tensor      # [B]
    seasons: Tuple[Tuple[float, int], ...]


def _features(ts: torch.Tensor, t0: torch.Tensor, span: torch.Tensor, cps: torch.Tensor,
              seasons) -> torch.Tensor:
    """ts [B, T] seconds → X [B, T, P]."""
    s = (ts - t0[:, None]) / span[:, None]
    hinge = torch.clamp(s[:, :, None] - cps[:, None, :], min=0.0)  # trend slope changes
    parts = [torch.stack([torch.ones_like(s), s], 2), hinge]
    for period, order in seasons:
        k = torch.arange(1, order + 1, dtype=ts.dtype, device=ts.device)
        ang = 2 * math.pi * (ts[:, :, None] / period) * k  # absolute time: phase-consistent across series
        parts += [torch.sin(ang), torch.cos(ang)]
    return torch.cat(parts, 2)


def fit_prophet(hist: torch.Tensor, hist_end: torch.Tensor, step: torch.Tensor, n_changepoints: int = 10,
                cp_range: float = 0.8, ridge_cp: float = 10.0, ridge: float = 1e-4) -> ProphetFit:
    """``hist [B, T]`` (NaN = missing; last sample at ``hist_end``, spacing ``step``)."""
    B, T = hist.shape
    dev = hist.device
    dt = torch.float64
    y = hist.to(dt)
    w = (~torch.isnan(y)).to(dt)
    y = torch.nan_to_num(y, nan=0.0)
    j = torch.arange(T, dtype=dt, device=dev)
    ts = hist_end.to(dt)[:, None] - (T - 1 - j)[None, :] * step.to(dt)[:, None]
    # first/last valid timestamps per series
    big = torch.tensor(float("inf"), dtype=dt, device=dev)
    t0 = torch.where(w > 0, ts, big).min(1).values
    t1 = torch.where(w > 0, ts, -big).max(1).values
    ok = torch.isfinite(t0) & (t1 > t0)
    t0 = torch.where(ok, t0, ts[:, 0])
    span = torch.where(ok, t1 - t0, torch.full_like(t0, 1.0))
    cps = (torch.arange(1, n_changepoints + 1, dtype=dt, device=dev) / (n_changepoints + 1) * cp_range)
    cps = cps[None, :].expand(B, -1).contiguous()
    span_max = float(span.max()) if B else 0.0
    seasons: List[Tuple[float, int]] = []
    if span_max >= 2 * DAY:
        seasons.append((DAY, 4))
    if span_max >= 2 * WEEK:
        seasons.append((WEEK, 3))
    X = _features(ts, t0, span, cps, seasons)  # [B, T, P]
    P = X.shape[2]
    ysc = torch.where(w > 0, y.abs(), torch.zeros_like(y)).max(1).values.clamp(min=1e-12)
    yn = y / ysc[:, None]
    Xw = X * w[:, :, None]
    A = Xw.transpose(1, 2) @ X  # [B, P, P]
    reg = torch.full((P,), ridge, dtype=dt, device=dev)
    reg[2:2 + n_changepoints] = ridge_cp
    A = A + torch.diag(reg)[None]
    rhs = (Xw.transpose(1, 2) @ yn[:, :, None])  # [B, P, 1]
    beta = torch.linalg.solve(A, rhs)[:, :, 0]
    r = (yn - (X @ beta[:, :, None])[:, :, 0]) * w
    n = w.sum(1)
    sigma = torch.sqrt((r * r).sum(1) / (n - P).clamp(min=1.0)) * ysc
    return ProphetFit(beta=beta, sigma=sigma.to(hist.dtype), n_valid=n.to(torch.int32), t0=t0, span=span,
                      cps=cps, yscale=ysc, seasons=tuple(seasons))


def forecast(fit: ProphetFit, ts: torch.Tensor) -> torch.Tensor:
    """``ts [B, C]`` absolute timestamps → forecast ``[B, C]``."""
    X = _features(ts.to(torch.float64), fit.t0, fit.span, fit.cps, fit.seasons)
    return ((X @ fit.beta[:, :, None])[:, :, 0] * fit.yscale[:, None]).to(torch.float32)
