"""Bivariate normal scorer (two metrics; ``docs/guides/design.md:78``).

Per series pair (e.g. latency and error rate of one app): fit the 2-D mean
and covariance on the historical window, score current points by squared
Mahalanobis distance ``d²``.  A point is anomalous when ``d² > thr²``
(``thr`` in sigma units, the same ``threshold`` env as the univariate
models).  Reference semantics for the ``bivariate`` kernel (K8).
"""

from __future__ import annotations

from dataclasses import dataclass

import torch


@dataclass
class BivariateFit:
    mean: torch.Tensor   # [N, 2]
    cov: torch.Tensor    # [N, 3] (sxx, sxy, syy)
    count: torch.Tensor  # [N]


def fit_bivariate(h: torch.Tensor) -> BivariateFit:
    """``h``: ``[N, T, 2]``; a time point is used only if both coordinates are valid."""
    h = h.float()
    valid = ~torch.isnan(h).any(2)
    n = valid.sum(1).float()
    z = torch.where(valid[..., None], h, torch.zeros_like(h))
    mean = z.sum(1) / n.clamp(min=1)[:, None]
    d = torch.where(valid[..., None], h - mean[:, None, :], torch.zeros_like(h))
    sxx = (d[..., 0] * d[..., 0]).sum(1) / n.clamp(min=1)
    sxy = (d[..., 0] * d[..., 1]).sum(1) / n.clamp(min=1)
    syy = (d[..., 1] * d[..., 1]).sum(1) / n.clamp(min=1)
    return BivariateFit(mean=mean, cov=torch.stack([sxx, sxy, syy], 1), count=n)


def mahalanobis2(fit: BivariateFit, x: torch.Tensor, eps: float = 1e-9) -> torch.Tensor:
    """``x``: ``[N, C, 2]`` → ``d² [N, C]`` (NaN where x is missing)."""
    x = x.float()
    sxx, sxy, syy = fit.cov[:, 0] + eps, fit.cov[:, 1], fit.cov[:, 2] + eps
    det = sxx * syy - sxy * sxy
    det = torch.where(det.abs() < 1e-20, torch.full_like(det, 1e-20), det)
    dx = x[..., 0] - fit.mean[:, None, 0]
    dy = x[..., 1] - fit.mean[:, None, 1]
    return (syy[:, None] * dx * dx - 2 * sxy[:, None] * dx * dy + sxx[:, None] * dy * dy) / det[:, None]
