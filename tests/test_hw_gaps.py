"""Holt-Winters variant 5 on gapped series (hw_scan.hip ``hw_dg_kernel``): a pair with a
missing observation past season 0 is fitted by the masked-season residual walk, not
the variant-4 general kernel.  Checked against the fp64 reference (models/smoothing.py:
a missing step carries the forecast, adds no SSE term and is not counted for sigma)."""

import numpy as np
import pytest
import torch

from foremast_amd.models import smoothing as sm_ref
from tests.test_kernels_gpu import _assert_near_optimal, _ref_detect, _ring, _series

pytestmark = pytest.mark.gpu

M = 1440
GRID = sm_ref.make_grid(sm_ref.MODE_HW, (0.1, 0.3, 0.5, 0.8), (0.0, 0.01, 0.05, 0.1), (0.05, 0.1, 0.3, 0.5))


@pytest.fixture(scope="module")
def K():
    from foremast_amd.ops import _native, kernels
    _native.require()
    return kernels


def _gapped(case, N, T, seed):
    """Series with production-shaped gaps: isolated scrape misses, a 30-minute outage,
    an outage across a season boundary, a whole missing season, and misses in the
    first / last fitted season (the pass-1 prologue and the non-fused last season)."""
    y = _series(N, T, M, seed=seed)
    rng = np.random.default_rng(seed + 1)
    if case == "miss1e-3":
        y[rng.random(y.shape) < 1e-3] = np.nan
    elif case == "miss1e-2":
        y[rng.random(y.shape) < 1e-2] = np.nan
    elif case == "outage30":
        for n in range(0, N, 2):                      # every other series: one 30-minute outage
            s = int(rng.integers(M, T - 30))
            y[n, s:s + 30] = np.nan
    elif case == "boundary":
        y[::3, 3 * M - 40:3 * M + 50] = np.nan       # across the season 2 / 3 boundary
        y[1::3, M - 5:M + 100] = np.nan              # season 0 / 1: season 1's pass 1
    elif case == "season":
        y[::4, 2 * M:3 * M] = np.nan                 # one whole fitted season missing
        y[1::4, T - 60:] = np.nan                    # the newest hour (last season)
        y[2::4, M:M + 45] = np.nan                   # exactly lane 0 of season 1
    elif case == "mixed":
        y[rng.random(y.shape) < 3e-3] = np.nan
        y[::5, 4000:4030] = np.nan
        y[::7, :200] = np.nan                        # season-0 gaps too
    return y


@pytest.mark.parametrize("case", ["miss1e-3", "miss1e-2", "outage30", "boundary", "season", "mixed"])
def test_gapped_pairs_match_reference(K, case):
    dev = torch.device("cuda:0")
    N, T = 18, 10080
    R, head = T + 64, 1064                             # aligned ring, head mid-ring: chunked staging
    y = _gapped(case, N, T, seed=len(case) * 13)
    ring = torch.tensor(_ring(y, R, head), device=dev).to(torch.bfloat16)
    yl = ring.float().cpu().numpy()[:, (head + np.arange(T)) % R]
    C = 50
    hz = torch.arange(1, 11, dtype=torch.int32).repeat(C // 10)
    cur = torch.tensor(np.nan_to_num(y[:, -C:], nan=20.0) * 1.05, device=dev)
    spec = K.DetectSpec(horizons=hz.to(dev), threshold=torch.full((N,), 2.0, device=dev),
                        bound=torch.full((N,), 3, dtype=torch.int8, device=dev),
                        min_lower=torch.full((N,), -1e30, device=dev), cur=cur, max_horizon=10)
    K.hw_clear_gap_flags()  # earlier cases of this size flagged other pairs
    before = K.hw_deferred_total(dev)
    out = K.smoothing_fit(ring, head, T, sm_ref.MODE_HW, M, GRID.to(dev), spec, variant=5, defer_detect=False)
    torch.cuda.synchronize()
    assert K.last_hw_variant == 5
    gapped_pairs = int(np.isnan(yl[:, M:]).reshape(N // 2, -1).any(1).sum())
    assert K.hw_deferred_total(dev) - before == gapped_pairs > 0
    # the next fit of the same data: the flagged pairs skip the dense kernel's staging and the
    # gapped kernel gives the same result bit for bit
    again = {k: v.clone() for k, v in K.smoothing_fit(ring, head, T, sm_ref.MODE_HW, M, GRID.to(dev), spec,
                                                      variant=5).items()}
    torch.cuda.synchronize()
    for key in ("best", "level", "trend", "sigma", "verdict", "forecast"):
        assert torch.equal(again[key], out[key]), key
    ref = sm_ref.fit_smoothing(torch.tensor(yl, dtype=torch.float64), sm_ref.MODE_HW, GRID.double(), m=M)
    kb = out["best"].cpu().long()
    same = (kb == ref.best).numpy()
    assert same.mean() >= 0.75
    _assert_near_optimal(yl, GRID, sm_ref.MODE_HW, M, kb)
    np.testing.assert_allclose(out["sigma"].cpu().numpy(), ref.sigma.numpy(), rtol=5e-3)
    np.testing.assert_allclose(out["level"].cpu().numpy()[same], ref.level.numpy()[same], rtol=2e-3, atol=5e-3)
    np.testing.assert_allclose(out["trend"].cpu().numpy()[same], ref.trend.numpy()[same], rtol=2e-2, atol=2e-4)
    f_ref = sm_ref.forecast(ref, hz.long())
    np.testing.assert_allclose(out["forecast"].cpu().numpy()[same], f_ref.numpy()[same], rtol=5e-3, atol=2e-2)
    d = _ref_detect(out, GRID, sm_ref.MODE_HW, M, hz, cur)
    assert torch.equal(d.count, out["count"].cpu())
    assert torch.equal(d.verdict, out["verdict"].cpu())


@pytest.mark.parametrize("case", ["miss1e-3", "outage30", "season"])
def test_gapped_deferred_detect_reports_valid_points(K, case):
    """defer_detect: the gapped kernel stores the series' valid-point count (sigma's
    denominator) for the split detection kernel, equal to the reference's."""
    dev = torch.device("cuda:0")
    N, T = 16, 10080
    y = _gapped(case, N, T, seed=7)
    ring = torch.tensor(y, device=dev).to(torch.bfloat16)
    yl = ring.float().cpu().numpy()
    C = 20
    hz = torch.arange(1, 11, dtype=torch.int32).repeat(2)
    cur = torch.tensor(np.nan_to_num(y[:, -C:], nan=20.0) * 1.05, device=dev)
    spec = K.DetectSpec(horizons=hz.to(dev), threshold=torch.full((N,), 2.0, device=dev),
                        bound=torch.full((N,), 3, dtype=torch.int8, device=dev),
                        min_lower=torch.full((N,), -1e30, device=dev), cur=cur, max_horizon=10)
    out = K.smoothing_fit(ring, 0, T, sm_ref.MODE_HW, M, GRID.to(dev), spec, variant=5, defer_detect=True)
    if K.last_detect_deferred:
        K.hw_detect_deferred(out, spec, T, M, grid=GRID.to(dev))
    torch.cuda.synchronize()
    ref = sm_ref.fit_smoothing(torch.tensor(yl, dtype=torch.float64), sm_ref.MODE_HW, GRID.double(), m=M)
    np.testing.assert_array_equal(out["nvalid"].cpu().numpy(), ref.n_valid.numpy())
    kb = out["best"].cpu().long()
    d = _ref_detect(out, GRID, sm_ref.MODE_HW, M, hz, cur)
    assert torch.equal(d.verdict, out["verdict"].cpu())
    assert (kb == ref.best).float().mean() >= 0.75


def test_gapped_pruning_is_exact(K, monkeypatch):
    """The grid branch and bound in the gapped kernel returns exactly the exhaustive fit."""
    dev = torch.device("cuda:0")
    N, T = 64, 10080
    y = _gapped("mixed", N, T, seed=3)
    y[4::9] = 7.0                                     # constant: every SSE ties
    y[4::9, 3000:3010] = np.nan
    ring = torch.tensor(y, device=dev).to(torch.bfloat16)
    hz = torch.arange(1, 11, dtype=torch.int32).repeat(5)
    cur = torch.tensor(np.nan_to_num(y[:, -50:], nan=20.0) * 1.04, device=dev)
    spec = K.DetectSpec(horizons=hz.to(dev), threshold=torch.full((N,), 2.0, device=dev),
                        bound=torch.full((N,), 3, dtype=torch.int8, device=dev),
                        min_lower=torch.full((N,), -1e30, device=dev), cur=cur, max_horizon=10)
    outs = []
    for prune in ("0", "1", "1"):                     # the second pruned run uses the winners as hints
        monkeypatch.setenv("FOREMAST_HW_PRUNE", prune)
        o = K.smoothing_fit(ring, 0, T, sm_ref.MODE_HW, M, GRID.to(dev), spec, variant=5,
                            out=outs[-1] if prune == "1" and len(outs) == 2 else None)
        torch.cuda.synchronize()
        outs.append({k: v.clone() for k, v in o.items()})
    for o in outs[1:]:
        for key in ("best", "level", "trend", "sigma", "verdict", "count", "forecast", "upper", "lower"):
            assert torch.equal(o[key], outs[0][key]), key


def test_gapped_kernel_agrees_with_general_kernel(K, monkeypatch):
    """Same input through the new gapped walk and the variant-4 general kernel
    (FOREMAST_HW_GAPS=v4): the same grid points, sigma to float rounding."""
    dev = torch.device("cuda:0")
    N, T = 40, 10080
    y = _gapped("mixed", N, T, seed=9)
    ring = torch.tensor(y, device=dev).to(torch.bfloat16)
    spec = K.DetectSpec(horizons=torch.arange(1, 11, dtype=torch.int32, device=dev),
                        threshold=torch.full((N,), 2.0, device=dev),
                        bound=torch.full((N,), 3, dtype=torch.int8, device=dev),
                        min_lower=torch.full((N,), -1e30, device=dev),
                        cur=torch.tensor(np.nan_to_num(y[:, -10:], nan=20.0), device=dev), max_horizon=10)
    outs = []
    for gaps in ("v5", "v4"):
        monkeypatch.setenv("FOREMAST_HW_GAPS", gaps)
        o = K.smoothing_fit(ring, 0, T, sm_ref.MODE_HW, M, GRID.to(dev), spec, variant=5)
        torch.cuda.synchronize()
        outs.append({k: v.clone() for k, v in o.items()})
    assert (outs[0]["best"] == outs[1]["best"]).float().mean() >= 0.9
    np.testing.assert_allclose(outs[0]["sigma"].cpu().numpy(), outs[1]["sigma"].cpu().numpy(), rtol=2e-3)


@pytest.mark.parametrize("case", ["dense", "miss1e-3", "outage"])
def test_variant5_at_the_300s_step_matches_reference(K, case, monkeypatch):
    """Variant 5 at the 300 s step (a daily season of 288 = 32 lanes x 9 steps, the week =
    2,016 points): the same fit as the fp64 reference, dense and gapped (the gapped kernel
    at K = 9), and the branch and bound exact."""
    dev = torch.device("cuda:0")
    m, N = 288, 22
    T = 7 * m
    y = _series(N, T, m, seed=41)
    rng = np.random.default_rng(42)
    if case == "miss1e-3":
        y[rng.random(y.shape) < 2e-3] = np.nan
    elif case == "outage":
        y[::3, 3 * m + 17:3 * m + 23] = np.nan           # 30 minutes = 6 points
    ring = torch.tensor(y, device=dev).to(torch.bfloat16)
    yl = ring.float().cpu().numpy()
    C = 8
    hz = torch.tensor([1, 2, 1, 2, 1, 2, 1, 2], dtype=torch.int32)
    cur = torch.tensor(np.nan_to_num(y[:, -C:], nan=20.0) * 1.05, device=dev)
    spec = K.DetectSpec(horizons=hz.to(dev), threshold=torch.full((N,), 2.0, device=dev),
                        bound=torch.full((N,), 3, dtype=torch.int8, device=dev),
                        min_lower=torch.full((N,), -1e30, device=dev), cur=cur, max_horizon=2)
    K.hw_clear_gap_flags()
    outs = []
    for prune in ("1", "0"):
        monkeypatch.setenv("FOREMAST_HW_PRUNE", prune)
        o = K.smoothing_fit(ring, 0, T, sm_ref.MODE_HW, m, GRID.to(dev), spec, variant=5)
        torch.cuda.synchronize()
        assert K.last_hw_variant == 5
        outs.append({k: v.clone() for k, v in o.items()})
    for key in ("best", "level", "trend", "sigma", "verdict", "forecast"):
        assert torch.equal(outs[0][key], outs[1][key]), key
    out = outs[0]
    ref = sm_ref.fit_smoothing(torch.tensor(yl, dtype=torch.float64), sm_ref.MODE_HW, GRID.double(), m=m)
    kb = out["best"].cpu().long()
    same = (kb == ref.best).numpy()
    assert same.mean() >= 0.75
    _assert_near_optimal(yl, GRID, sm_ref.MODE_HW, m, kb)
    np.testing.assert_allclose(out["sigma"].cpu().numpy(), ref.sigma.numpy(), rtol=5e-3)
    np.testing.assert_allclose(out["level"].cpu().numpy()[same], ref.level.numpy()[same], rtol=2e-3, atol=5e-3)
    f_ref = sm_ref.forecast(ref, hz.long())
    np.testing.assert_allclose(out["forecast"].cpu().numpy()[same], f_ref.numpy()[same], rtol=5e-3, atol=2e-2)
    d = _ref_detect(out, GRID, sm_ref.MODE_HW, m, hz, cur)
    assert torch.equal(d.verdict, out["verdict"].cpu())


@pytest.mark.parametrize("case", ["dense", "outage"])
def test_quad_kernel_matches_pair_kernel_at_300s(K, case, monkeypatch):
    """At m = 288 variant 5 walks four series per wave (hw_q_kernel, 16 lanes x 18 steps);
    FOREMAST_HW_QUAD=0 runs the 32-lane K = 9 kernel.  Same fits up to the summation order
    of the SSE (row vs half sums): the same grid point almost everywhere, sigma to float
    rounding.  The outage case defers gapped quads to the 32-lane gapped kernel.  N = 23
    leaves a partial quad (padding series)."""
    dev = torch.device("cuda:0")
    m, N = 288, 23
    T = 7 * m
    y = _series(N, T, m, seed=43)
    if case == "outage":
        y[::4, 2 * m + 100:2 * m + 106] = np.nan
    ring = torch.tensor(y, device=dev).to(torch.bfloat16)
    C = 10
    spec = K.DetectSpec(horizons=torch.arange(1, C + 1, dtype=torch.int32, device=dev),
                        threshold=torch.full((N,), 2.0, device=dev),
                        bound=torch.full((N,), 3, dtype=torch.int8, device=dev),
                        min_lower=torch.full((N,), -1e30, device=dev),
                        cur=torch.tensor(np.nan_to_num(y[:, -C:], nan=20.0) * 1.05, device=dev), max_horizon=C)
    K.hw_clear_gap_flags()
    outs = []
    for quad in ("1", "0"):
        monkeypatch.setenv("FOREMAST_HW_QUAD", quad)
        if quad == "0":
            # the 32-lane kernel takes horizons <= K = 9 only
            spec = K.DetectSpec(horizons=torch.arange(1, 10, dtype=torch.int32, device=dev),
                                threshold=spec.threshold, bound=spec.bound, min_lower=spec.min_lower,
                                cur=spec.cur[:, :9].contiguous(), max_horizon=9)
        o = K.smoothing_fit(ring, 0, T, sm_ref.MODE_HW, m, GRID.to(dev), spec, variant=5)
        torch.cuda.synchronize()
        assert K.last_hw_variant == 5
        outs.append({k: v.clone() for k, v in o.items()})
    assert (outs[0]["best"] == outs[1]["best"]).float().mean() >= 0.95
    same = (outs[0]["best"] == outs[1]["best"]).cpu().numpy()
    np.testing.assert_allclose(outs[0]["sigma"].cpu().numpy(), outs[1]["sigma"].cpu().numpy(), rtol=1e-3)
    np.testing.assert_allclose(outs[0]["level"].cpu().numpy()[same], outs[1]["level"].cpu().numpy()[same],
                               rtol=1e-4, atol=1e-3)
    # and against the fp64 reference
    ref = sm_ref.fit_smoothing(torch.tensor(ring.float().cpu().numpy(), dtype=torch.float64), sm_ref.MODE_HW,
                               GRID.double(), m=m)
    np.testing.assert_allclose(outs[0]["sigma"].cpu().numpy(), ref.sigma.numpy(), rtol=5e-3)


@pytest.mark.parametrize("case", ["miss", "outage"])
def test_quad_path_gapped_pairs_forecast_long_horizons(K, case):
    """At m = 288 the quad path takes forecast horizons up to 16 while its gapped pairs run the
    32-lane K = 9 gapped kernel: the seasonal phases 9..15 of a series come from the lane that
    owns them (lane 1).  Before the fix they were never written, so horizons >= 10 read stale
    LDS (the 300 s canary with isolated misses flagged 17,459 of 20,000 healthy apps)."""
    dev = torch.device("cuda:0")
    m, N = 288, 24
    T = 7 * m
    y = _series(N, T, m, seed=77)
    rng = np.random.default_rng(78)
    if case == "miss":
        y[rng.random(y.shape) < 2e-3] = np.nan
    else:
        y[::2, 4 * m + 30:4 * m + 36] = np.nan
    ring = torch.tensor(y, device=dev).to(torch.bfloat16)
    yl = ring.float().cpu().numpy()
    C = 16
    hz = torch.arange(1, C + 1, dtype=torch.int32)
    cur = torch.tensor(np.nan_to_num(y[:, -C:], nan=20.0), device=dev)
    spec = K.DetectSpec(horizons=hz.to(dev), threshold=torch.full((N,), 4.0, device=dev),
                        bound=torch.full((N,), 3, dtype=torch.int8, device=dev),
                        min_lower=torch.full((N,), -1e30, device=dev), cur=cur, max_horizon=C)
    K.hw_clear_gap_flags()
    before = K.hw_deferred_total(dev)
    out = K.smoothing_fit(ring, 0, T, sm_ref.MODE_HW, m, GRID.to(dev), spec, variant=5)
    torch.cuda.synchronize()
    assert K.last_hw_variant == 5 and K.hw_deferred_total(dev) > before   # gapped pairs took the K = 9 kernel
    ref = sm_ref.fit_smoothing(torch.tensor(yl, dtype=torch.float64), sm_ref.MODE_HW, GRID.double(), m=m)
    same = (out["best"].cpu().long() == ref.best).numpy()
    assert same.mean() >= 0.75
    f_ref = sm_ref.forecast(ref, hz.long())
    np.testing.assert_allclose(out["forecast"].cpu().numpy()[same], f_ref.numpy()[same], rtol=5e-3, atol=2e-2)
    d = _ref_detect(out, GRID, sm_ref.MODE_HW, m, hz, cur, thr=4.0)
    assert torch.equal(d.verdict, out["verdict"].cpu())
