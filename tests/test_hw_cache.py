"""Cached Holt-Winters model (``ShardSpec.refit_every``): state extraction after a
refit and O(1) per-tick state updates, CPU reference vs the gfx950 kernels
(ops/csrc/hw_state.hip)."""

import pytest
import torch

from foremast_amd.brain.engine import ShardSpec, StreamingShard, synthetic_history
from foremast_amd.models import smoothing as sm
from foremast_amd.utils.config import BrainConfig


def _grid():
    cfg = BrainConfig()
    return sm.make_grid(sm.MODE_HW, cfg.hw_alpha, cfg.hw_beta, cfg.hw_gamma)


def _series(n, T, m, seed=0, nan_frac=0.02):
    y = synthetic_history(n, T, m, torch.device("cpu"), seed=seed)
    g = torch.Generator().manual_seed(seed + 1)
    y[torch.rand(y.shape, generator=g) < nan_frac] = float("nan")
    return y


def test_hw_run_reproduces_the_fitted_state():
    """hw_run with each series' fitted grid point = the fit's best state."""
    n, m = 12, 24
    y = _series(n, 5 * m - 7, m)  # front padding of 7 steps
    grid = _grid()
    fit = sm.fit_smoothing(y, sm.MODE_HW, grid, m=m)
    st = sm.hw_run(y, grid[fit.best], m)
    assert st.t_last == fit.t_len - 1
    torch.testing.assert_close(st.level, fit.level, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(st.trend, fit.trend, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(st.season, fit.season, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(sm.hw_state_forecast(st, torch.arange(1, 6)), sm.forecast(fit, torch.arange(1, 6)),
                               rtol=1e-5, atol=1e-4)


def test_hw_update_equals_the_recursion_over_the_extended_series():
    n, m, k = 10, 24, 9
    y = _series(n, 4 * m + k, m, seed=5)
    T = 4 * m
    params = _grid()[torch.randint(0, 64, (n,), generator=torch.Generator().manual_seed(2))]
    st = sm.hw_run(y[:, :T], params, m)
    sm.hw_update(st, y[:, T:], params)
    ref = sm.hw_run(y, params, m, pad_to=T + k)
    assert st.t_last == ref.t_last
    torch.testing.assert_close(st.level, ref.level)
    torch.testing.assert_close(st.season, ref.season)


def _shard(dev, refit_every, n=16, R=None, m=48, P=3, W=4, seed=3, dtype=torch.float32):
    R = R or 5 * m
    cfg = BrainConfig()
    cfg.min_historical_points = 0
    sh = StreamingShard(ShardSpec(n_series=n, ring_len=R, season=m, pods=P, window=W, n_apps=4,
                                  refit_every=refit_every, dtype=dtype), cfg, dev,
                        app_id=(torch.arange(n, device=dev) % 4).int())
    hist = synthetic_history(n, R + 40, m, torch.device("cpu"), seed=seed).to(dev)
    sh.load_history(hist[:, :R])
    sh.set_baseline(hist[:, R - W:R].repeat(1, P).float())
    return sh, hist


def test_engine_cache_schedule_and_forecast_cpu():
    """refit_every=4: refit, 3 cached ticks, refit...; a cached tick's forecast is
    the fitted state advanced by every graduated point (oracle: hw_run over the
    refit window plus those points with the refit's grid points)."""
    dev = torch.device("cpu")
    sh, hist = _shard(dev, 4)
    R, m, P, W = sh.hist.R, sh.spec.season, sh.cur.P, sh.cur.W
    flags = []
    window0 = best = None
    for k in range(W + 9):
        sh.ingest_tick(hist[:, R + k:R + k + 1].repeat(1, P).float())
        out = sh.score()
        flags.append(sh.last_refit)
        if sh.last_refit:
            window0 = sh.hist.logical().float().clone()
            best = out["best"].long().clone()
            n_since = 0
        else:
            n_since += int(k >= W)  # a point graduates once the window is full
            ext = torch.cat([window0, sh.hist.logical().float()[:, R - n_since:]], 1)
            ref = sm.hw_run(ext, sh.grid[best], m, pad_to=R + n_since)
            f = sm.hw_state_forecast(ref, sh.horizons.long())
            torch.testing.assert_close(out["forecast"], f, rtol=1e-5, atol=1e-4)
    # the window fills for W ticks (no graduation), then the cache cycle starts
    steady = flags[W:]
    assert steady[:9] == [True, False, False, False, True, False, False, False, True]


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,pad", [(torch.float32, 0), (torch.bfloat16, 37)])
def test_hw_state_kernel_matches_reference(dtype, pad):
    from foremast_amd.ops import _native
    from foremast_amd.ops import kernels as K
    _native.require()
    dev = torch.device("cuda:0")
    n, m = 300, 128
    T = 5 * m - pad
    R = T + 50
    y = _series(n, T, m, seed=11)
    ring = torch.full((n, R), float("nan"))
    head = 77
    idx = (torch.arange(T) + head) % R
    ring[:, idx] = y
    ring = ring.to(dev, dtype)
    yq = ring.float().cpu()[:, idx]  # the values the kernel sees (bf16-rounded)
    grid = _grid()
    best = torch.randint(0, 64, (n,), generator=torch.Generator().manual_seed(4)).int()
    st = K.hw_state(ring, head, T, m, grid.to(dev), best.to(dev))
    ref = sm.hw_run(yq, grid[best.long()], m)
    assert st["Tp"] - 1 == ref.t_last
    torch.cuda.synchronize()
    torch.testing.assert_close(st["level"].cpu(), ref.level, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(st["trend"].cpu(), ref.trend, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(st["season"].cpu().T, ref.season, rtol=1e-4, atol=1e-3)
    nv = (~torch.isnan(torch.cat([torch.full((n, pad), float("nan")), yq], 1)[:, m:])).sum(1).float()
    assert torch.equal(st["nvalid"].cpu(), nv)


@pytest.mark.gpu
@pytest.mark.parametrize("refit_every", [1, 3])
def test_cached_engine_gpu_matches_cpu(refit_every):
    """GPU StreamingShard vs the CPU StreamingShard on the same data at m = 1440,
    P = 5, W = 10, pairwise ALL: refit every tick (variant-5 fit, side-stream rank
    tests, deferred band/verdict) or every 3 ticks (+ state kernel, update/detect
    kernel): refit schedule, verdicts, forecasts, app counters."""
    from foremast_amd.ops import _native
    _native.require()
    n, m, P, W = 64, 1440, 5, 10
    R = 3 * m
    cpu, hist = _shard(torch.device("cpu"), refit_every, n=n, R=R, m=m, P=P, W=W, seed=21)
    gpu, _ = _shard(torch.device("cuda:0"), refit_every, n=n, R=R, m=m, P=P, W=W, seed=21, dtype=torch.bfloat16)
    g = torch.Generator().manual_seed(7)
    for k in range(W + 7):
        newv = hist[:, R + k:R + k + 1].repeat(1, P).float() + 0.5 * torch.randn(n, P, generator=g)
        if k >= W + 3:
            newv[::9] *= 2.0
        outs = {}
        for sh in (cpu, gpu):
            sh.ingest_tick(newv.to(sh.device))
        # the GPU ring is bf16: score the CPU engine on the same rounded values
        cpu.hist.data.copy_(gpu.hist.data.float().cpu())
        for where, sh in (("cpu", cpu), ("cuda:0", gpu)):
            outs[where] = {key: v.detach().cpu().clone() for key, v in sh.score().items() if torch.is_tensor(v)}
        assert cpu.last_refit == gpu.last_refit, k
        o_c, o_g = outs["cpu"], outs["cuda:0"]
        torch.testing.assert_close(o_g["forecast"], o_c["forecast"], rtol=2e-3, atol=2e-2, msg=f"tick {k}")
        agree = (o_g["verdict"] == o_c["verdict"]).float().mean().item()
        assert agree >= 0.97, (k, agree)
        if agree == 1.0:
            assert torch.equal(cpu.app_stats, gpu.app_stats.cpu()), k
    assert (gpu._cache is not None) == (refit_every > 1)
