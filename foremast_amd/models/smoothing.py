"""Exponential smoothing family: ES, double ES (Holt), additive Holt-Winters.

The brain's single-metric models (``docs/guides/design.md:68-71``) as batched
PyTorch over ``[N, T]`` series.  This module is the *reference semantics*;
``foremast_amd.ops.smoothing_fit`` is the gfx950 kernel that must match it.

Recurrence (error-correction form, additive, season ``m``)::

    f_t = l + b                 (level+trend forecast)
    e_t = y_t - s[t mod m] - f_t
    l  <- f_t + alpha * e_t
    b  <- b + alpha * beta * e_t
    s[t mod m] <- s[t mod m] + gamma * (1 - alpha) * e_t
    SSE += e_t^2

which is algebraically identical to the textbook Holt-Winters update
(``l' = a(y-s) + (1-a)(l+b)``, ``b' = b(l'-l)+(1-b)b``, ``s' = g(y-l')+(1-g)s``).
Missing points (NaN) are imputed by the forecast (``e_t = 0``) and excluded
from the SSE.

Initialisation (design decision, docs/SCORING.md):

* HW: the series is front-padded with NaN to a multiple of ``m``; season 0
  initialises ``l0 = nanmean(season0)``, ``b0 = (nanmean(season1) - l0)/m``,
  ``s[p] = y[p] - l0`` (0 where missing); fitting runs over seasons 1..K-1.
* ES / DES: ``l0`` = first valid value, ``b0 = 0``; fitting runs over all t
  (the first valid point contributes e = 0 and counts as valid).

Parameters are fitted by exhaustive grid search (argmin SSE over the
``alpha x beta x gamma`` grid); ``sigma = sqrt(SSE / n_valid)``.
Forecast for horizon ``h >= 1`` after the last point ``T-1``:
``l_T + h b_T + s[(T-1+h) mod m]``.
"""

from __future__ import annotations

import itertools
from dataclasses import dataclass
from typing import Optional, Sequence

import torch

MODE_ES = 0
MODE_DES = 1
MODE_HW = 2

MODE_BY_NAME = {"exponential_smoothing": MODE_ES, "double_exponential_smoothing": MODE_DES,
                "holt_winters": MODE_HW}


@dataclass
class SmoothingFit:
    level: torch.Tensor      # [N]
    trend: torch.Tensor      # [N]
    season: Optional[torch.Tensor]  # [N, m] (phase-indexed, padded time)
    sigma: torch.Tensor      # [N]
    best: torch.Tensor       # [N] int64 grid index
    sse: torch.Tensor        # [N]
    n_valid: torch.Tensor    # [N]
    pad: int                 # front padding applied (HW)
    t_len: int               # padded length
    m: int


def make_grid(mode: int, alphas: Sequence[float], betas: Sequence[float],
              gammas: Sequence[float]) -> torch.Tensor:
    """Grid as ``[G, 3]`` (alpha, beta, gamma); unused axes collapse to 0."""
    if mode == MODE_ES:
        rows = [(a, 0.0, 0.0) for a in alphas]
    elif mode == MODE_DES:
        rows = [(a, b, 0.0) for a, b in itertools.product(alphas, betas)]
    else:
        rows = [(a, b, g) for a, b, g in itertools.product(alphas, betas, gammas)]
    return torch.tensor(rows, dtype=torch.float32)


def _nanmean(x: torch.Tensor, dim: int) -> torch.Tensor:
    v = ~torch.isnan(x)
    s = torch.where(v, x, torch.zeros_like(x)).sum(dim)
    n = v.sum(dim)
    return torch.where(n > 0, s / n.clamp(min=1), torch.zeros_like(s))


def padded_length(mode: int, T: int, m: int, chunk: int = 1) -> int:
    unit = m if mode == MODE_HW else chunk
    return ((T + unit - 1) // unit) * unit


def fit_smoothing(y: torch.Tensor, mode: int, grid: torch.Tensor, m: int = 1,
                  pad_to: Optional[int] = None) -> SmoothingFit:
    """Reference grid fit.  ``y``: ``[N, T]`` float; returns the best state."""
    y = y.float()
    N, T = y.shape
    dev = y.device
    G = grid.shape[0]
    if mode == MODE_HW:
        Tp = pad_to or padded_length(mode, T, m)
        if Tp // m < 2:
            raise ValueError(f"holt_winters needs >= 2 seasons (T={T}, m={m})")
    else:
        Tp = pad_to or T
        m = 1
    pad = Tp - T
    if pad:
        y = torch.cat([torch.full((N, pad), float("nan"), device=dev), y], dim=1)
    alpha = grid[:, 0].to(dev).view(1, G)
    beta = grid[:, 1].to(dev).view(1, G)
    gamma = grid[:, 2].to(dev).view(1, G)
    ab = alpha * beta
    g1a = gamma * (1.0 - alpha)

    if mode == MODE_HW:
        s0 = y[:, :m]
        l0 = _nanmean(s0, 1)
        l1 = _nanmean(y[:, m:2 * m], 1)
        b0 = (l1 - l0) / m
        season = torch.where(torch.isnan(s0), torch.zeros_like(s0), s0 - l0[:, None])
        season = season[:, None, :].expand(N, G, m).clone()
        t0 = m
    else:
        valid = ~torch.isnan(y)
        first_idx = torch.where(valid.any(1), valid.float().argmax(1), torch.zeros(N, dtype=torch.long, device=dev))
        l0 = y.gather(1, first_idx[:, None]).squeeze(1)
        l0 = torch.where(torch.isnan(l0), torch.zeros_like(l0), l0)
        b0 = torch.zeros_like(l0)
        season = None
        # t0 = 0: the first valid point has e = 0 by construction; padded /
        # leading NaN steps are no-ops because b0 = 0.
        t0 = 0
    lvl = l0[:, None].expand(N, G).clone()
    trd = b0[:, None].expand(N, G).clone()
    sse = torch.zeros(N, G, device=dev)
    nval = torch.zeros(N, device=dev)
    for t in range(t0, Tp):
        yt = y[:, t:t + 1]
        ok = ~torch.isnan(yt)
        if mode == MODE_HW:
            p = t % m
            s = season[:, :, p]
            e = yt - s - lvl - trd
        else:
            e = yt - lvl - trd
        e = torch.where(ok, e, torch.zeros_like(e))
        lvl = lvl + trd + alpha * e
        trd = trd + ab * e
        if mode == MODE_HW:
            season[:, :, p] = s + g1a * e
        sse = sse + e * e
        nval = nval + ok.squeeze(1).float()
    best = sse.argmin(1)
    idx = best[:, None]
    sse_b = sse.gather(1, idx).squeeze(1)
    sigma = torch.sqrt(sse_b / nval.clamp(min=1))
    seas_b = None
    if mode == MODE_HW:
        seas_b = season.gather(1, idx[:, :, None].expand(N, 1, m)).squeeze(1)
    return SmoothingFit(level=lvl.gather(1, idx).squeeze(1), trend=trd.gather(1, idx).squeeze(1),
                        season=seas_b, sigma=sigma, best=best, sse=sse_b, n_valid=nval,
                        pad=pad, t_len=Tp, m=m)


def forecast(fit: SmoothingFit, horizons: torch.Tensor) -> torch.Tensor:
    """``horizons``: ``[C]`` or ``[N, C]`` int (>= 1) → ``[N, C]`` forecasts."""
    h = horizons.to(fit.level.device)
    if h.dim() == 1:
        h = h[None, :].expand(fit.level.shape[0], -1)
    f = fit.level[:, None] + h.float() * fit.trend[:, None]
    if fit.season is not None:
        ph = (fit.t_len - 1 + h.long()) % fit.m
        f = f + fit.season.gather(1, ph)
    return f


# ---------------------------------------------------------------------------------
# Cached model (streaming engine ``refit_every > 1``; ops/csrc/hw_state.hip)
# ---------------------------------------------------------------------------------

@dataclass
class HwState:
    """State of a fitted Holt-Winters model after the point at padded time
    ``t_last``: forecast for horizon h is ``level + h trend + season[(t_last + h) mod m]``."""
    level: torch.Tensor   # [N]
    trend: torch.Tensor   # [N]
    season: torch.Tensor  # [N, m] (padded-time phase)
    t_last: int
    m: int


def hw_run(y: torch.Tensor, params: torch.Tensor, m: int, pad_to: Optional[int] = None) -> HwState:
    """The Holt-Winters recursion of :func:`fit_smoothing` with ONE parameter
    row per series (``params [N, 3]`` = alpha, beta, gamma; e.g. the fitted grid
    points), same initialisation and padding; returns the end state."""
    y = y.float()
    N, T = y.shape
    Tp = pad_to or padded_length(MODE_HW, T, m)
    pad = Tp - T
    if pad:
        y = torch.cat([torch.full((N, pad), float("nan"), device=y.device), y], dim=1)
    al, be, ga = (params[:, i].to(y.device).float() for i in range(3))
    ab, g1a = al * be, ga * (1.0 - al)
    s0 = y[:, :m]
    l0 = _nanmean(s0, 1)
    lvl = l0.clone()
    trd = (_nanmean(y[:, m:2 * m], 1) - l0) / m
    season = torch.where(torch.isnan(s0), torch.zeros_like(s0), s0 - l0[:, None])
    for t in range(m, Tp):
        p = t % m
        yt = y[:, t]
        e = torch.where(torch.isnan(yt), torch.zeros_like(yt), yt - season[:, p] - lvl - trd)
        lvl = lvl + trd + al * e
        trd = trd + ab * e
        season[:, p] = season[:, p] + g1a * e
    return HwState(level=lvl, trend=trd, season=season, t_last=Tp - 1, m=m)


def hw_update(st: HwState, y: torch.Tensor, params: torch.Tensor) -> HwState:
    """Advance the state by new points ``y [N, k]`` (oldest first; NaN = missing,
    imputed by the forecast) in place."""
    al, be, ga = (params[:, i].to(y.device).float() for i in range(3))
    ab, g1a = al * be, ga * (1.0 - al)
    for j in range(y.shape[1]):
        st.t_last += 1
        p = st.t_last % st.m
        yt = y[:, j].float()
        e = torch.where(torch.isnan(yt), torch.zeros_like(yt), yt - st.season[:, p] - st.level - st.trend)
        st.level = st.level + st.trend + al * e
        st.trend = st.trend + ab * e
        st.season[:, p] = st.season[:, p] + g1a * e
    return st


def hw_state_forecast(st: HwState, horizons: torch.Tensor) -> torch.Tensor:
    """``horizons [C]`` or ``[N, C]`` (>= 1) → ``[N, C]`` forecasts from the state."""
    h = horizons.to(st.level.device)
    if h.dim() == 1:
        h = h[None, :].expand(st.level.shape[0], -1)
    ph = (st.t_last + h.long()) % st.m
    return st.level[:, None] + h.float() * st.trend[:, None] + st.season.gather(1, ph)
