"""Band construction, anomaly detection and per-series verdicts (K9/K11).

Given a model forecast ``f [N, C]`` and spread ``sigma [N]`` for the current
window points ``x [N, C]``:

* pairwise adjustment (K11, ``docs/guides/design.md:35``): when the canary
  test says baseline and current differ, ``thr_eff = thr * pairwise_scale``
  (default 0.5, design decision);
* ``upper = f + thr_eff·sigma``;
  ``lower = max(f - thr_eff·sigma, min_lower_bound)``;
* ``bound``: 1 → anomaly iff ``x > upper``; 2 → iff ``x < lower``;
  3 → either (``foremast-brain/README.md:24``, design decision);
* verdict per series: ``1`` anomalous (any anomalous point), ``0`` healthy,
  ``-1`` unknown (no current point, or no model).
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


def detect(forecast: torch.Tensor, sigma: torch.Tensor, x: torch.Tensor,
           threshold: torch.Tensor, bound: torch.Tensor, min_lower: torch.Tensor,
           differs: Optional[torch.Tensor] = None, pairwise_scale: float = 0.5,
           model_ok: Optional[torch.Tensor] = None) -> Detection:
    f = forecast.float()
    N, C = f.shape
    thr = threshold.float().expand(N) if threshold.dim() == 0 else threshold.float()
    if differs is not None:
        thr = torch.where(differs.bool(), thr * pairwise_scale, thr)
    sig = sigma.float()
    upper = f + thr[:, None] * sig[:, None]
    lower = torch.maximum(f - thr[:, None] * sig[:, None], min_lower.float().view(-1, 1).expand(N, 1))
    xv = x.float()
    valid = ~torch.isnan(xv)
    bnd = bound.view(-1, 1).expand(N, 1).long()
    hi = (xv > upper) & ((bnd & 1) != 0)
    lo = (xv < lower) & ((bnd & 2) != 0)
    anom = (hi | lo) & valid
    if model_ok is not None:
        anom = anom & model_ok.view(-1, 1)
    count = anom.sum(1).to(torch.int32)
    has = valid.any(1)
    if model_ok is not None:
        has = has & model_ok
    verdict = torch.where(count > 0, torch.ones_like(count),
                          torch.where(has, torch.zeros_like(count), torch.full_like(count, -1)))
    z = torch.where(valid, (xv - f).abs() / sig[:, None].clamp(min=1e-12), torch.zeros_like(xv))
    return Detection(upper=upper, lower=lower, anomaly=anom, count=count,
                     verdict=verdict.to(torch.int8), score=z.amax(1))
