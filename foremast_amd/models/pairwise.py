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
* ``friedmanchisquare`` over ``[N, n_blocks, k]`` groups (``friedman``), and
  over time-slot blocks x pods of the canary windows (``friedman_pods``: the
  design doc's "Friedman chi-square (special case)", ``design.md:92``).

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
PW_FRIEDMAN = 6

PW_BY_NAME = {"NONE": PW_NONE, "ALL": PW_ALL, "ANY": PW_ANY, "MANN_WHITE": PW_MANN_WHITE,
              "MANN_WHITNEY": PW_MANN_WHITE, "WILCOXON": PW_WILCOXON, "KRUSKAL": PW_KRUSKAL,
              "FRIEDMAN": PW_FRIEDMAN}


def norm_sf(z: torch.Tensor) -> torch.Tensor:
    return 0.5 * torch.erfc(z / math.sqrt(2.0))


def _ranks_with_ties(x: torch.Tensor, valid: torch.Tensor):
    """Average ranks (1-based) among valid entries per row, and the tie term
    ``sum(t^3 - t)`` per row.  O(n^2) pairwise counting (exact for ties)."""
    big = torch.where(valid, x, torch.full_like(x, float("inf")))
    xi = big[:, :, None]
    xj = big[:, None, :]
    vj = valid[:, None, :]
    rt = torch.promote_types(x.dtype, torch.float32)
    less = ((xj < xi) & vj).sum(2).to(rt)
    eq = ((xj == xi) & vj).sum(2).to(rt)  # includes self
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
    p_friedman: Optional[torch.Tensor] = None
    n_blocks: Optional[torch.Tensor] = None


def friedman_pods(baseline: torch.Tensor, current: torch.Tensor, pods_b: int = 1, pods_c: int = 1):
    """Friedman chi-square with time slots as blocks and pods as treatments.

    ``baseline [N, pods_b * Wb]`` and ``current [N, pods_c * Wc]`` are pod-major
    windows whose slot j is the same time in every pod (the streaming engine's
    layout; the batch path pools pods, i.e. one pod per side).  Blocks are the
    first ``min(Wb, Wc)`` slots that are valid in every pod; ranks within a
    block, ties averaged, tie-corrected statistic, chi^2 with ``k - 1`` dof,
    ``k = pods_b + pods_c`` (scipy's ``friedmanchisquare`` over the complete
    blocks for k >= 3; k = 2 is the same statistic, which scipy refuses).
    Returns ``(p [N], complete blocks [N])``; no complete block gives p = 1."""
    dt = torch.promote_types(torch.promote_types(baseline.dtype, current.dtype), torch.float32)
    b = baseline.to(dt)
    c = current.to(dt)
    N, nb = b.shape
    nc = c.shape[1]
    Wb, Wc = nb // pods_b, nc // pods_c
    nbk = min(Wb, Wc)
    k = pods_b + pods_c
    g = torch.cat([b.reshape(N, pods_b, Wb)[:, :, :nbk], c.reshape(N, pods_c, Wc)[:, :, :nbk]], 1)
    g = g.transpose(1, 2)  # [N, blocks, k]
    ok = ~torch.isnan(g).any(2)
    flat = torch.nan_to_num(g, nan=0.0).reshape(N * nbk, k)
    r, tie = _ranks_with_ties(flat, torch.ones_like(flat, dtype=torch.bool))
    r = r.to(dt).reshape(N, nbk, k) * ok[..., None]
    tie = (tie.to(dt).reshape(N, nbk) * ok).sum(1)
    nblk = ok.sum(1).to(dt)
    Rj = r.sum(1)
    chi = 12.0 / (nblk * k * (k + 1)).clamp(min=1e-30) * (Rj * Rj).sum(1) - 3 * nblk * (k + 1)
    cc = 1 - tie / (nblk * k * (k * k - 1)).clamp(min=1e-30)
    chi = chi / cc.clamp(min=1e-30)
    p = torch.special.gammaincc(torch.full_like(chi, (k - 1) / 2.0), (chi / 2).clamp(min=0))
    p = torch.where((nblk > 0) & (cc > 0), p, torch.ones_like(p))
    return p, nblk


def rank_tests(baseline: torch.Tensor, current: torch.Tensor, pods=None) -> PairwiseResult:
    """All four tests; ``pods = (pods_b, pods_c)`` is the pod-major layout the
    Friedman test blocks on (default: one pod per side)."""
    dt = torch.promote_types(torch.promote_types(baseline.dtype, current.dtype), torch.float32)
    b = baseline.to(dt)
    c = current.to(dt)
    N, nb = b.shape
    nc = c.shape[1]
    x = torch.cat([b, c], 1)
    valid = ~torch.isnan(x)
    in_b = torch.zeros_like(valid)
    in_b[:, :nb] = True
    rank, tie = _ranks_with_ties(x, valid)
    n1 = valid[:, :nb].sum(1).to(dt)
    n2 = valid[:, nb:].sum(1).to(dt)
    n = n1 + n2
    R1 = torch.where(in_b, rank, torch.zeros_like(rank)).sum(1)
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
    # 12 / (n (n + 1)) sum R_i^2 / n_i - 3 (n + 1) without its cancellation: with
    # D = R1 - n1 (n + 1) / 2 = -(R2 - n2 (n + 1) / 2), H = 12 D^2 / ((n + 1) n1 n2)
    D = R1 - n1 * (n + 1) / 2
    H = 12.0 * D * D / ((n + 1) * n1 * n2).clamp(min=1)
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
    npairs = dvalid.sum(1).to(dt)
    Tplus = torch.where(dvalid & (d > 0), wr, torch.zeros_like(wr)).sum(1)
    Tminus = torch.where(dvalid & (d < 0), wr, torch.zeros_like(wr)).sum(1)
    Tw = torch.minimum(Tplus, Tminus)
    wmu = npairs * (npairs + 1) / 4
    wvar = npairs * (npairs + 1) * (2 * npairs + 1) / 24 - wtie / 48
    wsd = torch.sqrt(wvar.clamp(min=0))
    wz = (Tw - wmu) / wsd.clamp(min=1e-30)
    p_w = (2 * norm_sf(wz.abs())).clamp(max=1.0)
    p_w = torch.where((wsd > 0) & (npairs > 0), p_w, one)
    pb, pc = pods if pods is not None else (1, 1)
    p_fr, nblk = friedman_pods(baseline, current, pb, pc)
    return PairwiseResult(p_mw=p_mw, p_wilcoxon=p_w, p_kruskal=p_kw, n_base=n1, n_cur=n2,
                          n_pairs=npairs, p_friedman=p_fr, n_blocks=nblk)


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
                     min_wilcoxon: int = 20, min_kruskal: int = 5, min_friedman: int = 5) -> torch.Tensor:
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
    if mode == PW_FRIEDMAN:
        if res.p_friedman is None:
            raise ValueError("FRIEDMAN needs rank_tests(..., pods=...) results")
        return (res.n_blocks >= min_friedman) & (res.p_friedman < alpha)
    if mode == PW_ANY:
        return rej_mw | rej_w | rej_k
    any_ran = ran_mw | ran_w | ran_k
    ok_mw = ~ran_mw | rej_mw
    ok_w = ~ran_w | rej_w
    ok_k = ~ran_k | rej_k
    return any_ran & ok_mw & ok_w & ok_k
