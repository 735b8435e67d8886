"""Holt-Winters variant 6 (ops/csrc/hw_seq.hip): the sequential grid fit with the season in
registers, at the short daily seasons of the steps a create request may carry
(/root/reference/foremast-service/README.md:26-80; the 1200 s historical step sketched at
/root/reference/foremast-barrelman/pkg/client/metrics/metricsquery.go:74): m = 72 (1200 s),
24 (3600 s), 48 (1800 s), 96 (900 s), 144 (600 s).  Checked against the fp64 reference
(models/smoothing.py), with gaps (a missing step carries the forecast, adds no SSE term and
is not counted for sigma), front padding, a wrapped ring, the deferred detection, the device
ring head of graph replays and the variant-3 kernel on the same data."""

import numpy as np
import pytest
import torch

from foremast_amd.models import smoothing as sm_ref
from tests.test_kernels_gpu import _assert_near_optimal, _ref_detect, _ring, _series

pytestmark = pytest.mark.gpu

GRID = sm_ref.make_grid(sm_ref.MODE_HW, (0.1, 0.3, 0.5, 0.8), (0.0, 0.01, 0.05, 0.1), (0.05, 0.1, 0.3, 0.5))


@pytest.fixture(scope="module")
def K():
    from foremast_amd.ops import _native, kernels
    _native.require()
    return kernels


def _gapped(case, N, T, m, seed):
    y = _series(N, T, m, seed=seed)
    rng = np.random.default_rng(seed + 1)
    if case == "miss":
        y[rng.random(y.shape) < 5e-3] = np.nan          # isolated missed scrapes
    elif case == "outage":
        y[::2, 3 * m + 5:3 * m + 11] = np.nan            # 6 points across every other series
        y[1::3, m - 2:m + 3] = np.nan                    # across the season 0 / 1 boundary
    elif case == "season0":
        y[::3, :m // 2] = np.nan                         # half of season 0 (initialisation)
        y[1::5, m:2 * m] = np.nan                        # the whole of season 1 (b0 from nanmean 0)
        y[2::7, -4:] = np.nan                            # the newest points
    return y


def _spec(K, N, C, dev, y, hmax=10):
    hz = torch.arange(1, hmax + 1, dtype=torch.int32).repeat((C + hmax - 1) // hmax)[:C]
    cur = torch.tensor(np.nan_to_num(y[:, -C:], nan=20.0) * 1.05, device=dev)
    spec = K.DetectSpec(horizons=hz.to(dev), threshold=torch.full((N,), 2.0, device=dev),
                        bound=torch.full((N,), 3, dtype=torch.int8, device=dev),
                        min_lower=torch.full((N,), -1e30, device=dev), cur=cur, max_horizon=hmax)
    return spec, hz, cur


def _check(K, out, yl, m, hz, cur):
    ref = sm_ref.fit_smoothing(torch.tensor(yl, dtype=torch.float64), sm_ref.MODE_HW, GRID.double(), m=m)
    kb = out["best"].cpu().long()
    same = (kb == ref.best).numpy()
    assert same.mean() >= 0.75
    _assert_near_optimal(yl, GRID, sm_ref.MODE_HW, m, kb)
    np.testing.assert_allclose(out["sigma"].cpu().numpy(), ref.sigma.numpy(), rtol=5e-3)
    np.testing.assert_allclose(out["level"].cpu().numpy()[same], ref.level.numpy()[same], rtol=2e-3, atol=5e-3)
    np.testing.assert_allclose(out["trend"].cpu().numpy()[same], ref.trend.numpy()[same], rtol=2e-2, atol=2e-4)
    np.testing.assert_array_equal(out["nvalid"].cpu().numpy(), ref.n_valid.numpy())
    f_ref = sm_ref.forecast(ref, hz.long())
    np.testing.assert_allclose(out["forecast"].cpu().numpy()[same], f_ref.numpy()[same], rtol=5e-3, atol=2e-2)
    d = _ref_detect(out, GRID, sm_ref.MODE_HW, m, hz, cur)
    assert torch.equal(d.count, out["count"].cpu())
    assert torch.equal(d.verdict, out["verdict"].cpu())
    return ref, same


@pytest.mark.parametrize("case", ["dense", "miss", "outage", "season0"])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_seq_at_the_1200s_step_matches_reference(K, case, dtype):
    """m = 72 (a week = 504 points), a wrapped ring with the head mid-ring, a window that is
    not a whole number of seasons (front padding), N not a multiple of the series per
    workgroup (the last workgroup's rows past N)."""
    dev = torch.device("cuda:0")
    m, N = 72, 29
    T = 7 * m - 5
    R, head = T + 40, T - 20
    y = _gapped(case, N, T, m, seed=len(case) * 7)
    ring = torch.tensor(_ring(y, R, head), device=dev).to(dtype)
    yl = ring.float().cpu().numpy()[:, (head + np.arange(T)) % R]
    spec, hz, cur = _spec(K, N, 20, dev, y)
    out = K.smoothing_fit(ring, head, T, sm_ref.MODE_HW, m, GRID.to(dev), spec)
    torch.cuda.synchronize()
    assert K.last_hw_variant == 6
    _check(K, out, yl, m, hz, cur)


@pytest.mark.parametrize("m", [24, 48, 96, 144])
@pytest.mark.parametrize("case", ["dense", "miss"])
def test_seq_other_short_seasons_match_reference(K, m, case):
    dev = torch.device("cuda:0")
    N = 21
    T = 7 * m
    y = _gapped(case, N, T, m, seed=m)
    ring = torch.tensor(y, device=dev).to(torch.bfloat16)
    yl = ring.float().cpu().numpy()
    spec, hz, cur = _spec(K, N, 16, dev, y, hmax=16)
    out = K.smoothing_fit(ring, 0, T, sm_ref.MODE_HW, m, GRID.to(dev), spec)
    torch.cuda.synchronize()
    assert K.last_hw_variant == 6
    _check(K, out, yl, m, hz, cur)


@pytest.mark.parametrize("G", [1, 5, 16, 33])
def test_seq_small_and_odd_grids(K, G):
    """Grids of 1..64 points: two per thread (16 or 32 threads per series), the last thread's
    second point clamped onto the last one; the argmin over the series' threads."""
    dev = torch.device("cuda:0")
    m, N = 72, 13
    T = 6 * m
    grid = GRID[torch.randperm(GRID.shape[0], generator=torch.Generator().manual_seed(G))[:G]].contiguous()
    y = _gapped("miss", N, T, m, seed=G)
    ring = torch.tensor(y, device=dev)
    spec, hz, cur = _spec(K, N, 10, dev, y)
    out = K.smoothing_fit(ring, 0, T, sm_ref.MODE_HW, m, grid.to(dev), spec)
    torch.cuda.synchronize()
    assert K.last_hw_variant == 6
    ref = sm_ref.fit_smoothing(torch.tensor(y, dtype=torch.float64), sm_ref.MODE_HW, grid.double(), m=m)
    kb = out["best"].cpu().long()
    assert int(kb.max()) < G
    _assert_near_optimal(y, grid, sm_ref.MODE_HW, m, kb)
    np.testing.assert_allclose(out["sigma"].cpu().numpy(), ref.sigma.numpy(), rtol=5e-3)


def test_seq_deferred_detect_and_device_head(K):
    """defer_detect + hw_detect_deferred gives the inline epilogue's verdicts; the ring head
    read from a device scalar (HIP-graph replays) gives the host head's fit bit for bit."""
    dev = torch.device("cuda:0")
    m, N = 72, 40
    T = 7 * m
    R, head = T, 123                                    # a full ring (the graph tick's steady state)
    y = _gapped("miss", N, T, m, seed=5)
    ring = torch.tensor(_ring(y, R, head), device=dev).to(torch.bfloat16)
    spec, hz, cur = _spec(K, N, 10, dev, y)
    inline = {k: v.clone() for k, v in K.smoothing_fit(ring, head, T, sm_ref.MODE_HW, m, GRID.to(dev),
                                                        spec).items()}
    out = K.smoothing_fit(ring, 0, T, sm_ref.MODE_HW, m, GRID.to(dev), spec, defer_detect=True,
                          head_dev=torch.tensor([head], dtype=torch.int32, device=dev))
    assert K.last_hw_variant == 6 and K.last_detect_deferred
    K.hw_detect_deferred(out, spec, T, m, grid=GRID.to(dev))
    torch.cuda.synchronize()
    for key in ("best", "level", "trend", "sigma", "nvalid", "season_hb", "verdict", "count", "forecast",
                "upper", "lower"):
        assert torch.equal(out[key], inline[key]), key


def test_seq_season_output_and_variant3_agree(K, monkeypatch):
    """want_season: the winner's m seasonal terms, equal to the reference's where the grid
    point agrees; FOREMAST_HW_SEQ=0 runs the time-parallel variant 3 on the same data: the
    same grid points almost everywhere, sigma to float rounding."""
    dev = torch.device("cuda:0")
    m, N = 72, 24
    T = 7 * m
    y = _gapped("outage", N, T, m, seed=11)
    ring = torch.tensor(y, device=dev)
    spec, hz, cur = _spec(K, N, 10, dev, y)
    out = K.smoothing_fit(ring, 0, T, sm_ref.MODE_HW, m, GRID.to(dev), spec, want_season=True)
    torch.cuda.synchronize()
    assert K.last_hw_variant == 6
    ref = sm_ref.fit_smoothing(torch.tensor(y, dtype=torch.float64), sm_ref.MODE_HW, GRID.double(), m=m)
    same = (out["best"].cpu().long() == ref.best).numpy()
    np.testing.assert_allclose(out["season"].cpu().numpy()[same], ref.season.numpy()[same], rtol=5e-3, atol=5e-3)
    monkeypatch.setenv("FOREMAST_HW_SEQ", "0")
    v3 = K.smoothing_fit(ring, 0, T, sm_ref.MODE_HW, m, GRID.to(dev), spec, want_season=True)
    torch.cuda.synchronize()
    assert K.last_hw_variant == 3
    assert (v3["best"] == out["best"]).float().mean() >= 0.9
    np.testing.assert_allclose(v3["sigma"].cpu().numpy(), out["sigma"].cpu().numpy(), rtol=2e-3)


@pytest.mark.parametrize("case", ["dense", "miss", "outage"])
def test_seq_at_the_300s_step_matches_reference(K, case, monkeypatch):
    """Variant 6 at m = 288 (FOREMAST_HW_SEQ288=1): one grid point per thread, the 288 season
    registers partly in AGPRs (one wave per SIMD)."""
    monkeypatch.setenv("FOREMAST_HW_SEQ288", "1")
    dev = torch.device("cuda:0")
    m, N = 288, 9
    T = 7 * m
    y = _gapped(case, N, T, m, seed=288)
    ring = torch.tensor(y, device=dev).to(torch.bfloat16)
    yl = ring.float().cpu().numpy()
    spec, hz, cur = _spec(K, N, 10, dev, y)
    out = K.smoothing_fit(ring, 0, T, sm_ref.MODE_HW, m, GRID.to(dev), spec)
    torch.cuda.synchronize()
    assert K.last_hw_variant == 6
    _check(K, out, yl, m, hz, cur)


def test_batch_scorer_at_the_1200s_step_runs_variant6(K):
    """The per-job scorer (brain/batch.py, the service's jobs whose queries carry step 1200):
    the group's season is 86400 / 1200 = 72, so the GPU fit runs variant 6; its verdicts
    equal the CPU reference scorer's on the same tasks (x3 regressions in some canary
    windows, isolated misses in the histories)."""
    from foremast_amd.brain.batch import BatchScorer, MetricTask
    from foremast_amd.utils.config import BrainConfig
    step, m, T, C = 1200.0, 72, 504, 10
    N = 24
    y = _gapped("miss", N, T + C, m, seed=1200)
    base = _series(N, T + C, m, seed=77)[:, T:]
    cfg = BrainConfig()
    cfg.algorithm = "holt_winters"
    cfg.min_historical_points = 0
    t_end = 1_700_000_000.0
    tasks = []
    for i in range(N):
        cur = y[i, T:].copy()
        cur[np.isnan(cur)] = 20.0
        if i % 6 == 0:
            cur *= 3.0                                   # injected regression
        tasks.append(MetricTask(job_id=f"j{i}", alias="latency", metric="latency", namespace="ns", app=f"a{i}",
                                step=step, hist=y[i, :T].astype(np.float32), hist_end=t_end,
                                cur_ts=t_end + step * np.arange(1, C + 1), cur_vals=cur.astype(np.float32),
                                base_vals=base[i].astype(np.float32), threshold=3.0, bound=3))
    gpu = BatchScorer(cfg, device=torch.device("cuda:0")).score(tasks)
    torch.cuda.synchronize()
    assert K.last_hw_variant == 6
    cpu = BatchScorer(cfg, device=torch.device("cpu")).score(tasks)
    vg = np.array([r.verdict for r in gpu])
    vc = np.array([r.verdict for r in cpu])
    assert (vg == vc).mean() >= 0.95, (vg, vc)
    assert (vg[::6] == 1).all()
