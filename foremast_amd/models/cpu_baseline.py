"""CPU per-series baseline: the reference brain's design, measured.

The reference's brain (``intuit/foremast-brain``, not in the repository) is a
Python service that scores one job — one series — at a time on a 100m-CPU
budget (``deploy/foremast/3_brain/foremast-brain.yaml:82-86``).  This module is
that design re-created with the same scoring semantics as this repo's GPU
engine, as a per-series numpy/scipy loop, so "beats the reference" has an
anchor measured on the same synthetic data:

* Holt-Winters (additive, daily season, 7-day history): the 64-point
  alpha/beta/gamma grid fit, vectorised across the grid in numpy, sequential
  over time (the recurrence is what a per-series CPU brain runs);
* pairwise canary tests with scipy: ``mannwhitneyu``, ``wilcoxon``,
  ``kruskal`` (ML_PAIRWISE_ALGORITHM=ALL);
* band / verdict: h-step forecast sigma, Sidak window correction, lowered
  pairwise band with a minimum point count (``models/detect.py``).

``bench.py --config cpu_baseline`` times it single-threaded on a sample of the
benchmark's series; the per-core rate is the ``vs_baseline`` denominator.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np
from scipy import stats

from . import detect as det


@dataclass
class CpuVerdict:
    verdict: int
    count: int
    differs: bool
    best: int
    sigma: float


def hw_fit(y: np.ndarray, m: int, grid: np.ndarray):
    """One series' Holt-Winters grid fit (same recurrence and initialisation as
    ``models/smoothing.py``): returns (level, trend, season [m], sigma, best)."""
    T = len(y)
    Tp = ((T + m - 1) // m) * m
    if Tp // m < 2:
        raise ValueError("holt_winters needs >= 2 seasons")
    yp = np.concatenate([np.full(Tp - T, np.nan, dtype=np.float64), y.astype(np.float64)])
    a, b, g = grid[:, 0].astype(np.float64), grid[:, 1].astype(np.float64), grid[:, 2].astype(np.float64)
    ab, g1a = a * b, g * (1.0 - a)
    s0 = yp[:m]
    l0 = np.nanmean(s0)
    b0 = (np.nanmean(yp[m:2 * m]) - l0) / m
    season = np.repeat(np.where(np.isnan(s0), 0.0, s0 - l0)[:, None], len(grid), axis=1)  # [m, G]
    lvl = np.full(len(grid), l0)
    trd = np.full(len(grid), b0)
    sse = np.zeros(len(grid))
    nval = 0
    for t in range(m, Tp):
        yt = yp[t]
        if yt != yt:  # missing: the forecast stands in (e = 0)
            lvl = lvl + trd
            continue
        p = t % m
        s = season[p]
        e = yt - s - lvl - trd
        lvl = lvl + trd + a * e
        trd = trd + ab * e
        season[p] = s + g1a * e
        sse += e * e
        nval += 1
    k = int(np.argmin(sse))
    return lvl[k], trd[k], season[:, k].copy(), float(np.sqrt(sse[k] / max(nval, 1))), k, Tp


def score_series(hist: np.ndarray, cur: np.ndarray, base: Optional[np.ndarray], horizons: np.ndarray, m: int,
                 grid: np.ndarray, threshold: float = 4.0, bound: int = 3, alpha: float = 0.05,
                 pairwise_scale: float = 0.5, pw_min_points: int = 3, min_mw: int = 20, min_w: int = 20,
                 min_k: int = 5, shift_threshold: float = 0.0, shift_min_points: int = 1,
                 shift_one_step: bool = False) -> CpuVerdict:
    """Score ONE series: pairwise tests, HW fit, forecast, band, verdict."""
    differs = False
    if base is not None:
        c, bs = cur[~np.isnan(cur)], base[~np.isnan(base)]
        rej = []
        if min(len(c), len(bs)) >= min_mw:
            rej.append(stats.mannwhitneyu(bs, c, alternative="two-sided").pvalue < alpha)
        k = min(len(cur), len(base))
        d = cur[:k] - base[:k]
        d = d[~np.isnan(d)]
        if np.count_nonzero(d) >= min_w:
            rej.append(stats.wilcoxon(d).pvalue < alpha)
        if min(len(c), len(bs)) >= min_k:
            rej.append(stats.kruskal(bs, c).pvalue < alpha)
        differs = bool(rej) and all(rej)
    lvl, trd, season, sigma, best, Tp = hw_fit(hist, m, grid)
    f = lvl + horizons * trd + season[(Tp - 1 + horizons) % m]
    import torch
    kf = det.horizon_sigma_factor(torch.tensor(grid[best:best + 1]), 2, m, torch.tensor(horizons))[0].numpy()
    s = sigma * kf
    thr = torch.tensor([threshold])
    bnd = torch.tensor([bound])
    full = float(det.window_threshold(thr, bnd, len(cur))[0])
    low = float(det.window_threshold(thr * pairwise_scale, bnd, len(cur))[0])

    def outside(t):
        hi = (cur > f + t * s) if bound & 1 else np.zeros(len(cur), bool)
        lo = (cur < f - t * s) if bound & 2 else np.zeros(len(cur), bool)
        return int(np.count_nonzero((hi | lo) & ~np.isnan(cur)))

    n_full, n_low = outside(full), outside(low)
    count = n_low if (differs and n_low >= pw_min_points) else n_full
    ok = ~np.isnan(cur)
    bm = float(np.nanmean(base)) if base is not None and np.any(~np.isnan(base)) else float("nan")
    if (shift_threshold > 0 and differs and bm == bm and n_full == 0 and not n_low >= pw_min_points
            and np.count_nonzero(ok) >= max(shift_min_points, 1)):
        # the mean-shift rule (models/detect.py): canary window against the baseline mean, in
        # units of the one-step sigma (shift_one_step) or of the horizon-scaled band sigma
        ss = np.full(len(cur), sigma) if shift_one_step else s
        mz = float(np.mean((cur[ok] - bm) / np.maximum(ss[ok], 1e-12)))
        if ((bound & 1) and mz > shift_threshold) or ((bound & 2) and mz < -shift_threshold):
            hi = (cur > bm + shift_threshold * ss) if bound & 1 else np.zeros(len(cur), bool)
            lo = (cur < bm - shift_threshold * ss) if bound & 2 else np.zeros(len(cur), bool)
            count = int(np.count_nonzero((hi | lo) & ok))
    return CpuVerdict(verdict=1 if count else 0, count=count, differs=differs, best=best, sigma=sigma)
