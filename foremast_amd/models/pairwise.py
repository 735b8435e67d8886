"""Pairwise (baseline vs current) rank tests — Mann-Whitney U, Wilcoxon
signed-rank, Kruskal-Wallis, Friedman chi-square.

The brain's canary check (``docs/guides/design.md:35,89-92``;
``foremast-brain/README.md:34-38``): "if current and baseline have a
different distribution pattern, the threshold is lowered".

Batched over series: ``baseline [N, nb]``, ``current [N, nc]`` with NaN
padding.  Semantics match scipy's asymptotic forms (the oracle in
``tests/test_pairwise.py``):

* ``mannwhitneyu(b, c, alternative='two-sided', use_continuity=True,
  method='asymptotic')`` — tie-corrected normal approximation;
* ``wilcoxon(b[:k], c[:k], zero_method='wilcox', correction=False,
  method='approx')`` over the first ``k = min(nb, nc)`` aligned pairs where
  both are valid;
* ``kruskal(b, c)`` — tie-corrected H, chi² with 1 dof;
* ``friedmanchisquare`` over ``[N, n_blocks, k]`` groups.

Degenerate inputs (all values tied, too few points) give ``p = 1``
("no evidence of a difference"); min-point gates are the
``MIN_*_DATA_POINTS`` env values (``foremast-brain.yaml:74-79``).
"""

from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Optional

import torch

TEST_MW = 0
TEST_WILCOXON = 1
TEST_KRUSKAL = 2

# pairwise decision modes
PW_NONE = 0
PW_ALL = 1
PW_ANY = 2
PW_MANN_WHITE = 3
PW_WILCOXON = 4
PW_KRUSKAL = 5

PW_BY_NAME = {"NONE": PW_NONE, "ALL": PW_ALL, "ANY": PW_ANY, "MANN_WHITE": PW_MANN_WHITE,
              "MANN_WHITNEY": PW_MANN_WHITE, "WILCOXON": PW_WILCOXON, "KRUSKAL": PW_KRUSKAL,
              "FRIEDMAN": PW_KRUSKAL}


def norm_sf(z: torch.Tensor) -> torch.Tensor:
    return 0.5 * torch.erfc(z / math.sqrt(2.0))


def _ranks_with_ties(x: torch.Tensor, valid: torch.Tensor):
    """Average ranks (1-based) among valid entries per row, and the tie term
    ``sum(t^3 - t)`` per row.  O(n^2) pairwise counting (exact for ties)."""
    big = torch.where(valid, x, torch.full_like(x, float("inf")))
    xi = big[:, :, None]
    xj = big[:, None, :]
    vj = valid[:, None, :]
    less = ((xj < xi) & vj).sum(2).float()
    eq = ((xj == xi) & vj).sum(2).float()  # includes self
    rank = less + (eq + 1.0) / 2.0
    rank = torch.where(valid, rank, torch.zeros_like(rank))
    # sum over elements of (t_i^2 - 1) equals sum over tie groups of (t^3 - t)
    tie = torch.where(valid, eq * eq - 1.0, torch.zeros_like(eq)).sum(1)
    return rank, tie


@dataclass
class PairwiseResult:
    p_mw: torch.Tensor
    p_wilcoxon: torch.Tensor
    p_kruskal: torch.Tensor
    n_base: torch.Tensor
    n_cur: torch.Tensor
    n_pairs: torch.Tensor


def rank_tests(baseline: torch.Tensor, current: torch.Tensor) -> PairwiseResult:
    b = baseline.float()
    c = current.float()
    N, nb = b.shape
    nc = c.shape[1]
    x = torch.cat([b, c], 1)
    valid = ~torch.isnan(x)
    in_b = torch.zeros_like(valid)
    in_b[:, :nb] = True
    rank, tie = _ranks_with_ties(x, valid)
    n1 = valid[:, :nb].sum(1).float()
    n2 = valid[:, nb:].sum(1).float()
    n = n1 + n2
    R1 = torch.where(in_b, rank, torch.zeros_like(rank)).sum(1)
    R2 = torch.where(~in_b, rank, torch.zeros_like(rank)).sum(1)
    one = torch.ones_like(n)

    # --- Mann-Whitney U -----------------------------------------------------------
    U1 = R1 - n1 * (n1 + 1) / 2
    U2 = n1 * n2 - U1
    U = torch.maximum(U1, U2)
    mu = n1 * n2 / 2
    var = n1 * n2 / 12 * ((n + 1) - tie / (n * (n - 1)).clamp(min=1))
    sd = torch.sqrt(var.clamp(min=0))
    z = (U - mu - 0.5) / sd.clamp(min=1e-30)
    p_mw = (2 * norm_sf(z)).clamp(max=1.0)
    p_mw = torch.where((sd > 0) & (n1 > 0) & (n2 > 0), p_mw, one)

    # --- Kruskal-Wallis (2 groups) ------------------------------------------------
    H = 12.0 / (n * (n + 1)).clamp(min=1) * (R1 * R1 / n1.clamp(min=1) + R2 * R2 / n2.clamp(min=1)) \
        - 3 * (n + 1)
    corr = 1 - tie / (n * n * n - n).clamp(min=1)
    Hc = H / corr.clamp(min=1e-30)
    p_kw = torch.erfc(torch.sqrt(Hc.clamp(min=0) / 2))
    p_kw = torch.where((corr > 0) & (n1 > 0) & (n2 > 0), p_kw.clamp(max=1.0), one)

    # --- Wilcoxon signed rank over aligned pairs ---------------------------------
    k = min(nb, nc)
    d = c[:, :k] - b[:, :k]
    dvalid = ~torch.isnan(d) & (d != 0)
    ad = torch.where(dvalid, d.abs(), torch.zeros_like(d))
    wr, wtie = _ranks_with_ties(ad, dvalid)
    npairs = dvalid.sum(1).float()
    Tplus = torch.where(dvalid & (d > 0), wr, torch.zeros_like(wr)).sum(1)
    Tminus = torch.where(dvalid & (d < 0), wr, torch.zeros_like(wr)).sum(1)
    Tw = torch.minimum(Tplus, Tminus)
    wmu = npairs * (npairs + 1) / 4
    wvar = npairs * (npairs + 1) * (2 * npairs + 1) / 24 - wtie / 48
    wsd = torch.sqrt(wvar.clamp(min=0))
    wz = (Tw - wmu) / wsd.clamp(min=1e-30)
    p_w = (2 * norm_sf(wz.abs())).clamp(max=1.0)
    p_w = torch.where((wsd > 0) & (npairs > 0), p_w, one)
    return PairwiseResult(p_mw=p_mw, p_wilcoxon=p_w, p_kruskal=p_kw, n_base=n1, n_cur=n2,
                          n_pairs=npairs)


def friedman(groups: torch.Tensor) -> torch.Tensor:
    """Friedman chi-square over ``[N, n_blocks, k]`` (k >= 3 treatments);
    ranks within each block (ties averaged), tie-corrected, chi² with k-1 dof."""
    g = groups.float()
    N, nblk, k = g.shape
    flat = g.reshape(N * nblk, k)
    valid = torch.ones_like(flat, dtype=torch.bool)
    r, tie = _ranks_with_ties(flat, valid)
    r = r.reshape(N, nblk, k)
    tie = tie.reshape(N, nblk).sum(1)
    Rj = r.sum(1)  # [N, k]
    chi = 12.0 / (nblk * k * (k + 1)) * (Rj * Rj).sum(1) - 3 * nblk * (k + 1)
    c = 1 - tie / (nblk * k * (k * k - 1))
    chi = chi / c.clamp(min=1e-30)
    p = torch.special.gammaincc(torch.tensor((k - 1) / 2.0, device=g.device), (chi / 2).clamp(min=0))
    return torch.where(c > 0, p, torch.ones_like(p))


def pairwise_differs(res: PairwiseResult, mode: int, alpha: float, min_mw: int = 20,
                     min_wilcoxon: int = 20, min_kruskal: int = 5) -> torch.Tensor:
    """Decision: do baseline and current differ?  A test whose min-point gate
    is not met abstains.  ALL = every non-abstaining test rejects (and at least
    one ran); ANY = some test rejects."""
    n_small = torch.minimum(res.n_base, res.n_cur)
    ran_mw = n_small >= min_mw
    ran_w = res.n_pairs >= min_wilcoxon
    ran_k = n_small >= min_kruskal
    rej_mw = ran_mw & (res.p_mw < alpha)
    rej_w = ran_w & (res.p_wilcoxon < alpha)
    rej_k = ran_k & (res.p_kruskal < alpha)
    if mode == PW_NONE:
        return torch.zeros_like(ran_mw)
    if mode == PW_MANN_WHITE:
        return rej_mw
    if mode == PW_WILCOXON:
        return rej_w
    if mode == PW_KRUSKAL:
        return rej_k
    if mode == PW_ANY:
        return rej_mw | rej_w | rej_k
    any_ran = ran_mw | ran_w | ran_k
    ok_mw = ~ran_mw | rej_mw
    ok_w = ~ran_w | rej_w
    ok_k = ~ran_k | rej_k
    return any_ran & ok_mw & ok_w & ok_k
