"""Band construction, anomaly detection and per-series verdicts (K9/K11).

Given a model forecast ``f [N, C]`` and spread ``sigma`` for the current
window points ``x [N, C]``:

* spread per horizon: ``s = sigma * k(h)`` with ``k`` the h-step
  forecast-error factor of the fitted smoothing model
  (:func:`horizon_sigma_factor`; 1 for the moving average) — the band is a
  prediction interval for the horizon, not the one-step residual spread;
* window correction (:func:`window_threshold`, ``FOREMAST_WINDOW_CORRECTION``,
  default ``sidak``): ``threshold`` is the z-level at which a *window* of ``C``
  points is declared anomalous, so the per-point level is Sidak-adjusted
  (``P(any of C points outside) = P(one point outside at threshold)``); with
  ``none`` it is used per point unchanged;
* ``upper = f + thr·s``; ``lower = max(f - thr·s, min_lower_bound)``;
  ``bound``: 1 → anomaly iff ``x > upper``; 2 → iff ``x < lower``;
  3 → either (``foremast-brain/README.md:24``, design decision);
* pairwise adjustment (K11, ``docs/guides/design.md:35``): when the canary
  test says baseline and current differ, a second, lowered band
  (``threshold * pairwise_scale``, window-corrected the same way) applies —
  but only when at least ``pw_min_points`` points fall outside it
  (``ML_PAIRWISE_MIN_ANOMALIES``); a single point outside the full band is
  always an anomaly (fail fast on spikes);
* mean-shift rule (``shift_threshold`` > 0, ``ML_PAIRWISE_SHIFT``, needs
  ``base_mean``, the baseline pods' window mean): when the canary test says the
  pods differ and neither band fired, the series is anomalous if the canary
  window's mean deviation from the baseline mean, ``mean((x - base_mean) / s)``
  (at least ``shift_min_points`` points), is beyond ``shift_threshold`` on a side
  enabled by ``bound`` -- the rank tests' evidence of a level shift, sized
  against the model's spread.  Its band is ``base_mean +- shift_threshold * s``
  and its count the points outside it.  Measured against the baseline pods (not
  the forecast), it is immune to forecast bias: healthy canaries sit on their
  baseline whatever the model's error;
* verdict per series: ``1`` anomalous, ``0`` healthy, ``-1`` unknown (no
  current point, or no model).  ``upper``/``lower`` are the band of the rule
  in force (lowered band only when it fired).
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch

VERDICT_UNKNOWN = -1
VERDICT_HEALTHY = 0
VERDICT_ANOMALY = 1


@dataclass
class Detection:
    upper: torch.Tensor      # [N, C]
    lower: torch.Tensor      # [N, C]
    anomaly: torch.Tensor    # [N, C] bool
    count: torch.Tensor      # [N] int32
    verdict: torch.Tensor    # [N] int8
    score: torch.Tensor      # [N] max |x - f| / sigma over valid points


def norm_sf(x: torch.Tensor) -> torch.Tensor:
    return 0.5 * torch.erfc(x / 2 ** 0.5)


def window_threshold(threshold: torch.Tensor, bound: torch.Tensor, n_points, correction: str = "sidak") -> torch.Tensor:
    """Per-point z-level so that a window of ``n_points`` points exceeds it (on
    the sides enabled by ``bound``) with the probability a single point exceeds
    ``threshold``: ``p1 = sides * sf(thr)``, ``p = 1 - (1 - p1)^(1/C)``,
    ``z = isf(p / sides)`` (Sidak).  ``n_points``: int or ``[N]``."""
    thr = threshold.double()
    if correction == "none":
        return threshold.float()
    if correction != "sidak":
        raise ValueError(f"unknown window correction {correction!r}")
    n = torch.as_tensor(n_points, dtype=torch.float64, device=thr.device).expand_as(thr).clamp(min=1)
    sides = torch.where(bound.to(thr.device).long() == 3, 2.0, 1.0).double().expand_as(thr)
    p1 = (sides * norm_sf(thr)).clamp(1e-300, 1 - 1e-16)
    pc = -torch.expm1(torch.log1p(-p1) / n)
    z = -torch.special.ndtri((pc / sides).clamp(min=1e-300))
    z = torch.where(n <= 1, thr, z)
    return z.float()


def effective_thresholds(threshold: torch.Tensor, bound: torch.Tensor, n_points, pairwise_scale: float = 0.5,
                         correction: str = "sidak"):
    """(full, lowered) per-point thresholds ``[N]`` for :func:`detect` and the
    fused kernel epilogue (``DetectSpec.threshold`` / ``threshold_low``)."""
    thr = threshold.float()
    return (window_threshold(thr, bound, n_points, correction),
            window_threshold(thr * pairwise_scale, bound, n_points, correction))


def horizon_sigma_factor(params: torch.Tensor, mode: int, m: int, horizons: torch.Tensor) -> torch.Tensor:
    """``[N, C]`` factor ``k(h) = sqrt(v(h))`` of the h-step forecast error of the
    fitted smoothing model (``models/smoothing.py`` error-correction form,
    ``l += a e``, ``b += a b' e``, ``s += g (1 - a) e``)::

        v(h) = 1 + sum_{j=1}^{h-1} c_j^2,  c_j = a (1 + j b') + g (1 - a) [m > 0, j mod m == 0]

    ``params``: ``[N, 3]`` (alpha, beta, gamma) of the chosen grid point;
    ``mode``: 0 ES (b' = 0), 1 DES, 2 HW (season ``m``).  Same closed form as
    ``detect.h hstep_factor``."""
    p = params.double()
    a = p[:, 0:1]
    b = p[:, 1:2] if mode >= 1 else torch.zeros_like(a)
    h = horizons.double()
    if h.dim() == 1:
        h = h[None, :]
    hm1 = (h - 1).clamp(min=0)
    s1 = 0.5 * hm1 * h
    s2 = hm1 * h * (2 * h - 1) / 6
    v = 1 + a * a * (hm1 + 2 * b * s1 + b * b * s2)
    if mode == 2 and m > 0:
        g = p[:, 2:3] * (1 - a)
        k = torch.floor(hm1 / m)
        v = v + k * g * g + 2 * g * a * (k + m * b * 0.5 * k * (k + 1))
    v = torch.where(h <= 1, torch.ones_like(v), v)
    return torch.sqrt(v).float()


def detect(forecast: torch.Tensor, sigma: torch.Tensor, x: torch.Tensor,
           threshold: torch.Tensor, bound: torch.Tensor, min_lower: torch.Tensor,
           differs: Optional[torch.Tensor] = None, pairwise_scale: float = 0.5,
           model_ok: Optional[torch.Tensor] = None, threshold_low: Optional[torch.Tensor] = None,
           pw_min_points: int = 1, shift_threshold: float = 0.0,
           base_mean: Optional[torch.Tensor] = None, shift_min_points: int = 1,
           shift_sigma: Optional[torch.Tensor] = None) -> Detection:
    """``sigma``: ``[N]`` or per point ``[N, C]`` (horizon-scaled).  ``threshold``
    / ``threshold_low`` are per-point levels (already window-corrected, see
    :func:`effective_thresholds`); ``threshold_low`` defaults to
    ``threshold * pairwise_scale``.  ``shift_sigma`` (``[N]``, optional): the spread of
    the mean-shift rule (the model's one-step sigma, config ``pairwise_shift_one_step``);
    default ``sigma``."""
    f = forecast.float()
    N, C = f.shape
    thr = threshold.float().expand(N) if threshold.dim() == 0 else threshold.float()
    thr_low = thr * pairwise_scale if threshold_low is None else threshold_low.float()
    sig = sigma.float()
    sig = sig[:, None].expand(N, C) if sig.dim() == 1 else sig
    mlow = min_lower.float().view(-1, 1).expand(N, 1)
    xv = x.float()
    valid = ~torch.isnan(xv)
    bnd = bound.view(-1, 1).expand(N, 1).long()
    ok = torch.ones(N, dtype=torch.bool, device=f.device) if model_ok is None else model_ok.view(-1).bool()

    def outside(t):
        up = f + t[:, None] * sig
        lo = torch.maximum(f - t[:, None] * sig, mlow)
        an = (((xv > up) & ((bnd & 1) != 0)) | ((xv < lo) & ((bnd & 2) != 0))) & valid & ok[:, None]
        return up, lo, an

    up_f, lo_f, an_f = outside(thr)
    up_l, lo_l, an_l = outside(thr_low)
    cnt_f = an_f.sum(1)
    cnt_l = an_l.sum(1)
    dif = torch.zeros(N, dtype=torch.bool, device=f.device) if differs is None else differs.bool()
    low_rule = dif & (cnt_l >= max(int(pw_min_points), 1))
    shift_rule = torch.zeros_like(low_rule)
    use_shift = shift_threshold > 0 and base_mean is not None
    if use_shift:
        bm = base_mean.float().to(f.device).view(-1, 1)
        st = float(shift_threshold)
        ss = sig if shift_sigma is None else shift_sigma.float().to(f.device).view(-1, 1).expand(N, C)
        up_s = bm + st * ss
        lo_s = torch.maximum(bm - st * ss, mlow)
        an_s = (((xv > up_s) & ((bnd & 1) != 0)) | ((xv < lo_s) & ((bnd & 2) != 0))) & valid & ok[:, None]
        zb = torch.where(valid & ok[:, None], (xv - bm) / ss.clamp(min=1e-12), torch.zeros_like(xv))
        nz = (valid & ok[:, None]).sum(1)
        mz = zb.sum(1) / nz.clamp(min=1)
        side = (((bnd[:, 0] & 1) != 0) & (mz > st)) | (((bnd[:, 0] & 2) != 0) & (mz < -st))
        shift_rule = (dif & ~torch.isnan(bm[:, 0]) & ~low_rule & (cnt_f == 0)
                      & (nz >= max(int(shift_min_points), 1)) & side)
    lr, sr = low_rule[:, None], shift_rule[:, None]
    upper = torch.where(lr, up_l, up_f)
    lower = torch.where(lr, lo_l, lo_f)
    anom = torch.where(lr, an_l, an_f)
    count = torch.where(low_rule, cnt_l, cnt_f)
    if use_shift:
        upper, lower = torch.where(sr, up_s, upper), torch.where(sr, lo_s, lower)
        anom = torch.where(sr, an_s, anom)
        count = torch.where(shift_rule, an_s.sum(1), count)
    count = count.to(torch.int32)
    has = valid.any(1) & ok
    verdict = torch.where(count > 0, torch.ones_like(count),
                          torch.where(has, torch.zeros_like(count), torch.full_like(count, -1)))
    z = torch.where(valid, (xv - f).abs() / sig.clamp(min=1e-12), torch.zeros_like(xv))
    return Detection(upper=upper, lower=lower, anomaly=anom, count=count,
                     verdict=verdict.to(torch.int8), score=z.amax(1))
