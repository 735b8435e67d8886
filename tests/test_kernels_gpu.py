"""Numerics of the gfx950 kernels against the fp32 PyTorch references."""

import numpy as np
import pytest
import torch

from foremast_amd.models import bivariate as biv_ref
from foremast_amd.models import detect as det_ref
from foremast_amd.models import moving_average as ma_ref
from foremast_amd.models import pairwise as pw_ref
from foremast_amd.models import smoothing as sm_ref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def K():
    from foremast_amd.ops import _native, kernels
    _native.require()
    return kernels


def _series(N, T, m, seed=0, nan_frac=0.0):
    rng = np.random.default_rng(seed)
    t = np.arange(T)
    amp = rng.uniform(1, 5, (N, 1))
    lvl = rng.uniform(5, 50, (N, 1))
    slope = rng.uniform(-0.01, 0.01, (N, 1))
    y = lvl + slope * t + amp * np.sin(2 * np.pi * t / m + rng.uniform(0, 6, (N, 1))) \
        + rng.normal(0, 0.3, (N, T))
    if nan_frac:
        mask = rng.random((N, T)) < nan_frac
        y[mask] = np.nan
    return y.astype(np.float32)


def _ring(y, R, head):
    """Place logical series y [N, T] into a ring [N, R] starting at column head."""
    N, T = y.shape
    ring = np.full((N, R), 7.0, dtype=np.float32)
    cols = (head + np.arange(T)) % R
    ring[:, cols] = y
    return ring


def _det_spec(K, N, C, dev, cur=None, thr=2.0, bound=3):
    return K.DetectSpec(
        horizons=torch.arange(1, C + 1, dtype=torch.int32, device=dev),
        threshold=torch.full((N,), thr, device=dev), bound=torch.full((N,), bound, dtype=torch.int8, device=dev),
        min_lower=torch.full((N,), -1e30, device=dev), cur=cur)


def _ref_detect(out, grid, mode, m, hz, cur, thr=2.0, bound=3, differs=None, thr_low=None, pw_min=1):
    """Reference verdicts for a kernel fit: the kernel's own forecast and grid
    choice, sigma scaled to each horizon (models/detect.py horizon_sigma_factor)."""
    N = cur.shape[0]
    params = grid.cpu().float()[out["best"].cpu().long()]
    sig = out["sigma"].cpu()[:, None] * det_ref.horizon_sigma_factor(params, mode, m, hz.cpu())
    return det_ref.detect(out["forecast"].cpu(), sig, cur.cpu(), torch.full((N,), thr),
                          torch.full((N,), bound, dtype=torch.int8), torch.full((N,), -1e30),
                          differs=None if differs is None else differs.cpu(), threshold_low=thr_low,
                          pw_min_points=pw_min)


def _assert_near_optimal(yl, grid, mode, m, best, rel=1e-3):
    """The kernel's grid point must be within ``rel`` of the best fp64 SSE (bf16 /
    fp32 summation order may flip near-ties, but never pick a clearly worse fit)."""
    y64 = torch.tensor(yl, dtype=torch.float64)
    sse = torch.stack([sm_ref.fit_smoothing(y64, mode, grid[g:g + 1].double(), m=m).sse
                       for g in range(grid.shape[0])], 1)
    chosen = sse.gather(1, best.cpu().long()[:, None]).squeeze(1)
    opt = sse.min(1).values
    assert torch.all(chosen <= opt * (1 + rel) + 1e-6), (chosen / opt).max()


@pytest.mark.parametrize("mode,m,T,nan", [
    (sm_ref.MODE_HW, 24, 24 * 5 + 7, 0.0),
    (sm_ref.MODE_HW, 24, 24 * 6, 0.02),
    (sm_ref.MODE_HW, 100, 100 * 4, 0.0),
    (sm_ref.MODE_ES, 1, 3000, 0.0),
    (sm_ref.MODE_DES, 1, 2500, 0.01),
])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("variant", [-1, 0, 2, 3])
def test_smoothing_kernel_matches_reference(K, mode, m, T, nan, dtype, variant):
    dev = torch.device("cuda:0")
    N, C = 48, 12
    y = _series(N, T, max(m, 24), seed=T + mode, nan_frac=nan)
    R, head = T + 37, 29
    ring = torch.tensor(_ring(y, R, head), device=dev).to(dtype)
    yl = ring.float().cpu().numpy()[:, (head + np.arange(T)) % R]  # bf16-rounded logical
    grid = sm_ref.make_grid(mode, (0.1, 0.3, 0.6), (0.0, 0.05), (0.1, 0.4))
    cur = torch.tensor(y[:, -C:] * 1.05, device=dev)
    spec = _det_spec(K, N, C, dev, cur=cur)
    out = K.smoothing_fit(ring, head, T, mode, m, grid.to(dev), spec, want_season=True, variant=variant)
    torch.cuda.synchronize()
    ref = sm_ref.fit_smoothing(torch.tensor(yl, dtype=torch.float64), mode, grid.double(), m=m)
    # the kernel's chosen combo must be (near-)optimal under the reference SSE
    ref_all = []
    for g in range(grid.shape[0]):
        fg = sm_ref.fit_smoothing(torch.tensor(yl, dtype=torch.float64), mode, grid[g:g + 1].double(), m=m)
        ref_all.append(fg.sse)
    sse_all = torch.stack(ref_all, 1)  # [N, G]
    kb = out["best"].cpu().long()
    chosen = sse_all.gather(1, kb[:, None]).squeeze(1)
    assert torch.all(chosen <= ref.sse * (1 + 1e-4) + 1e-6), "kernel picked a sub-optimal grid point"
    same = kb == ref.best
    assert same.float().mean() > 0.9
    np.testing.assert_allclose(out["sigma"].cpu().numpy()[same.numpy()], ref.sigma.numpy()[same.numpy()],
                               rtol=2e-3, atol=1e-4)
    np.testing.assert_allclose(out["level"].cpu().numpy()[same.numpy()], ref.level.numpy()[same.numpy()],
                               rtol=1e-3, atol=2e-3)
    f_ref = sm_ref.forecast(ref, torch.arange(1, C + 1))
    np.testing.assert_allclose(out["forecast"].cpu().numpy()[same.numpy()], f_ref.numpy()[same.numpy()],
                               rtol=2e-3, atol=5e-3)
    d = _ref_detect(out, grid, mode, m, torch.arange(1, C + 1), cur)
    assert torch.equal(d.count, out["count"].cpu())
    assert torch.equal(d.verdict, out["verdict"].cpu())


@pytest.mark.parametrize("mode,T,nan,lead,N", [
    (sm_ref.MODE_ES, 3000, 0.0, 0, 300),     # last workgroup shifted back (300 % 128 != 0)
    (sm_ref.MODE_DES, 2500, 0.01, 0, 300),
    (sm_ref.MODE_ES, 777, 0.05, 150, 300),   # first chunks all missing for some series
    (sm_ref.MODE_DES, 10080, 0.0, 0, 300),
    (sm_ref.MODE_ES, 500, 0.02, 0, 50),      # N < series per workgroup: range-checked rows
])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_es_sequential_kernel_matches_reference(K, mode, T, nan, lead, N, dtype):
    """K2 sequential ES / DES (csrc/es_seq.hip): same argmin, sigma, level/trend,
    forecast and verdicts as the fp64 reference, through leading gaps and a ring
    that wraps."""
    dev = torch.device("cuda:0")
    C = 12
    y = _series(N, T, 24, seed=T + 7 * mode, nan_frac=nan)
    if lead:
        y[::3, :lead] = np.nan
    R, head = T + 37, 29
    ring = torch.tensor(_ring(y, R, head), device=dev).to(dtype)
    yl = ring.float().cpu().numpy()[:, (head + np.arange(T)) % R]
    grid = sm_ref.make_grid(mode, (0.1, 0.3, 0.6, 0.9), (0.0, 0.05, 0.1, 0.2), (0.0,))
    cur = torch.tensor(y[:, -C:] * 1.05, device=dev)
    spec = _det_spec(K, N, C, dev, cur=cur)
    out = K.smoothing_fit(ring, head, T, mode, 1, grid.to(dev), spec, variant=5)
    torch.cuda.synchronize()
    ref = sm_ref.fit_smoothing(torch.tensor(yl, dtype=torch.float64), mode, grid.double())
    kb = out["best"].cpu().long()
    same = (kb == ref.best).numpy()
    assert same.mean() > 0.97
    np.testing.assert_allclose(out["sigma"].cpu().numpy()[same], ref.sigma.numpy()[same], rtol=2e-3, atol=1e-4)
    np.testing.assert_allclose(out["level"].cpu().numpy()[same], ref.level.numpy()[same], rtol=1e-3, atol=2e-3)
    np.testing.assert_allclose(out["trend"].cpu().numpy()[same], ref.trend.numpy()[same], rtol=1e-2, atol=1e-4)
    np.testing.assert_allclose(out["nvalid"].cpu().numpy(), ref.n_valid.numpy())
    f_ref = sm_ref.forecast(ref, torch.arange(1, C + 1))
    np.testing.assert_allclose(out["forecast"].cpu().numpy()[same], f_ref.numpy()[same], rtol=2e-3, atol=5e-3)
    d = _ref_detect(out, grid, mode, 1, torch.arange(1, C + 1), cur)
    assert torch.equal(d.count, out["count"].cpu()) and torch.equal(d.verdict, out["verdict"].cpu())


@pytest.mark.parametrize("variant", [-1, 0, 1, 2, 3])
def test_smoothing_kernel_flagship_shape(K, variant):
    """T = 10080 (7 days at 60 s), season 1440 (daily), bf16 ring."""
    dev = torch.device("cuda:0")
    N, T, m, C = 16, 10080, 1440, 50
    y = _series(N, T, m, seed=5)
    ring = torch.tensor(y, device=dev).to(torch.bfloat16)
    grid = sm_ref.make_grid(sm_ref.MODE_HW, (0.1, 0.3, 0.5, 0.8), (0.0, 0.01, 0.05, 0.1), (0.05, 0.1, 0.3, 0.5))
    spec = _det_spec(K, N, C, dev, cur=torch.tensor(y[:, :C], device=dev))
    out = K.smoothing_fit(ring, 0, T, sm_ref.MODE_HW, m, grid.to(dev), spec, want_season=True, variant=variant)
    torch.cuda.synchronize()
    ref = sm_ref.fit_smoothing(ring.float().cpu(), sm_ref.MODE_HW, grid, m=m)
    same = (out["best"].cpu().long() == ref.best)
    assert same.float().mean() >= 0.75
    _assert_near_optimal(ring.float().cpu().numpy(), grid, sm_ref.MODE_HW, m, out["best"])
    np.testing.assert_allclose(out["sigma"].cpu().numpy(), ref.sigma.numpy(), rtol=5e-3)
    sm_ = same.numpy()
    np.testing.assert_allclose(out["season"].cpu().numpy()[sm_], ref.season.numpy()[sm_], rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("N", [40, 41, 43])  # a partial last workgroup (4 series per workgroup)
def test_window_stats_kernel(K, N):
    dev = torch.device("cuda:0")
    T, C = 1000, 8
    y = _series(N, T, 24, seed=11, nan_frac=0.05)
    for dtype in (torch.float32, torch.bfloat16):
        R, head = 1024, 1000  # wraps
        ring = torch.tensor(_ring(y, R, head), device=dev).to(dtype)
        yl = ring.float().cpu()[:, (head + np.arange(T)) % R]
        cur = torch.tensor(y[:, :C] + 3.0, device=dev)
        spec = _det_spec(K, N, C, dev, cur=cur)
        out = K.window_stats(ring, head, T, spec)
        torch.cuda.synchronize()
        st = ma_ref.window_stats(yl)
        np.testing.assert_allclose(out["mean"].cpu().numpy(), st.mean.numpy(), rtol=1e-5, atol=1e-4)
        np.testing.assert_allclose(out["std"].cpu().numpy(), st.std.numpy(), rtol=1e-4, atol=1e-4)
        d = det_ref.detect(st.mean[:, None].expand(N, C), st.std, cur.cpu(), torch.full((N,), 2.0),
                           torch.full((N,), 3, dtype=torch.int8), torch.full((N,), -1e30))
        assert torch.equal(d.verdict, out["verdict"].cpu())


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_window_stats_short_window_odd_head_and_offset(K, dtype):
    """A window shorter than the 64-lane wave starting at an unaligned head that wraps
    (the scalar head/tail path of the staged loads), and a large offset with a small
    variance (1e4 + N(0, 1e-2): cancellation in the per-lane shifted sums + Chan merge)."""
    dev = torch.device("cuda:0")
    N, R, L, head, C = 41, 1024, 60, 1001, 6
    rng = np.random.default_rng(3)
    y = (1e4 + rng.normal(0, 1e-2, (N, L))).astype(np.float32)
    y[::5, 7] = np.nan
    ring = torch.tensor(_ring(y, R, head), device=dev).to(dtype)
    yl = ring.float().cpu()[:, (head + np.arange(L)) % R]
    cur = torch.tensor(y[:, :C], device=dev)
    cur[::3, 2] += 1.0
    spec = _det_spec(K, N, C, dev, cur=cur, thr=3.0)
    out = K.window_stats(ring, head, L, spec)
    torch.cuda.synchronize()
    ref = torch.tensor(yl.numpy().astype(np.float64))
    ok = ~torch.isnan(ref)
    cnt = ok.sum(1)
    mean = torch.where(ok, ref, torch.zeros_like(ref)).sum(1) / cnt
    var = (torch.where(ok, ref - mean[:, None], torch.zeros_like(ref)) ** 2).sum(1) / cnt
    np.testing.assert_allclose(out["mean"].cpu().numpy(), mean.numpy(), rtol=1e-7, atol=2e-3)
    if dtype == torch.float32:  # bf16 quantises 1e4 + 1e-2 noise to a few levels: variance checked in fp32
        np.testing.assert_allclose(out["std"].cpu().numpy(), var.sqrt().numpy(), rtol=5e-2, atol=2e-3)
    assert torch.equal(out["count_hist"].cpu(), cnt.float())
    d = det_ref.detect(out["mean"].cpu()[:, None].expand(N, C), out["std"].cpu(), cur.cpu(), torch.full((N,), 3.0),
                       torch.full((N,), 3, dtype=torch.int8), torch.full((N,), -1e30))
    assert torch.equal(d.verdict, out["verdict"].cpu()) and torch.equal(d.count, out["count"].cpu())
    np.testing.assert_allclose(out["score"].cpu().numpy(), d.score.numpy(), rtol=1e-4)


def test_rank_tests_kernel(K):
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(3)
    N, nb, nc = 300, 50, 40
    b = rng.normal(0, 1, (N, nb)).astype(np.float32)
    c = (rng.normal(0, 1, (N, nc)) + rng.choice([0, 0.8], (N, 1))).astype(np.float32)
    b[::7] = np.round(b[::7])
    c[::7] = np.round(c[::7])
    b[5, 30:] = np.nan
    c[9, :4] = b[9, :4]
    out = K.rank_tests(torch.tensor(b, device=dev), torch.tensor(c, device=dev), pw_ref.PW_ALL, 0.05)
    torch.cuda.synchronize()
    ref = pw_ref.rank_tests(torch.tensor(b, dtype=torch.float64), torch.tensor(c, dtype=torch.float64))
    p = out["pvals"].cpu().double()
    np.testing.assert_allclose(p[:, 0].numpy(), ref.p_mw.numpy(), rtol=2e-3, atol=1e-5)
    np.testing.assert_allclose(p[:, 1].numpy(), ref.p_wilcoxon.numpy(), rtol=2e-3, atol=1e-5)
    np.testing.assert_allclose(p[:, 2].numpy(), ref.p_kruskal.numpy(), rtol=2e-3, atol=1e-5)
    dref = pw_ref.pairwise_differs(ref, pw_ref.PW_ALL, 0.05)
    agree = (out["differs"].cpu().bool() == dref).float().mean()
    assert agree > 0.99
    # the baseline window means (the mean-shift rule's centre)
    np.testing.assert_allclose(out["base_mean"].cpu().numpy(), np.nanmean(b, 1), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("nb,nc", [(55, 55), (64, 37), (20, 64)])
def test_rank_small_path_equals_sweep(K, nb, nc, monkeypatch):
    """The small-window path (sorted keys, run scans, one cross search) against the O(n^2)
    sweep on heavy ties, signed zeros, negative values, NaN gaps and partly filled canary
    windows: identical counts and decisions, p-values equal to fp32 rounding, and the
    decisions-only form (|z| > z_crit) identical to the p-value decisions."""
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(7)
    N = 4000
    b = torch.randn(N, nb, generator=g)
    c = torch.randn(N, nc, generator=g) + (torch.rand(N, 1, generator=g) < 0.3) * 0.7
    b[: N // 2] = torch.round(b[: N // 2] * 3) / 3        # heavy ties, many exact zeros
    c[: N // 2] = torch.round(c[: N // 2] * 3) / 3
    c[::5] = -c[::5]                                      # -0.0 next to +0.0
    fill = torch.randint(1, nc + 1, (N,), generator=g)
    c[torch.arange(nc)[None, :] >= fill[:, None]] = float("nan")
    b[torch.rand(N, nb, generator=g) < 0.05] = float("nan")
    c[3, :] = b[3, :nc] if nc <= nb else c[3, :]          # all pairs tied: no Wilcoxon pairs
    tb, tc = b.to(dev).contiguous(), c.to(dev).contiguous()
    outs = {}
    for path in ("small", "sweep"):
        if path == "sweep":
            monkeypatch.setenv("FOREMAST_RANK_SWEEP", "1")
        else:
            monkeypatch.delenv("FOREMAST_RANK_SWEEP", raising=False)
        for pv in (True, False):
            o = {}
            K.rank_tests(tb, tc, pw_ref.PW_ALL, 0.05, want_pvals=pv, out=o)
            outs[path, pv] = {k: v.clone() for k, v in o.items()}
    torch.cuda.synchronize()
    sm, sw = outs["small", True], outs["sweep", True]
    assert torch.equal(sm["counts"], sw["counts"])
    np.testing.assert_allclose(sm["pvals"].cpu().numpy(), sw["pvals"].cpu().numpy(), rtol=1e-5, atol=1e-6)
    assert torch.equal(sm["differs"], sw["differs"])
    assert torch.equal(outs["small", False]["differs"], sm["differs"])
    assert torch.equal(outs["sweep", False]["differs"], sw["differs"])
    # the reference on the same fp32 windows (c - b rounds in fp32 as in the kernel, so the
    # Wilcoxon ties are the same), its statistics exact and its tails in fp32
    ref = pw_ref.rank_tests(b, c)
    dref = pw_ref.pairwise_differs(ref, pw_ref.PW_ALL, 0.05)
    assert torch.equal(sm["differs"].cpu().bool(), dref)
    want = torch.stack([ref.p_mw, ref.p_wilcoxon, ref.p_kruskal], 1)
    ok = torch.isfinite(want)
    assert float((sm["pvals"].cpu().double()[ok] - want[ok]).abs().max()) < 2e-4


def test_rank_tests_kernel_friedman(K):
    """Friedman mode (time slots x pods) against the reference, with ties,
    incomplete blocks and a shifted canary."""
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(4)
    N, P, W = 257, 5, 10
    b = rng.normal(0, 1, (N, P * W)).astype(np.float32)
    c = (rng.normal(0, 1, (N, P * W)) + rng.choice([0, 1.0], (N, 1))).astype(np.float32)
    b[::5] = np.round(b[::5])
    c[::5] = np.round(c[::5])
    b[7, 3] = np.nan
    c[11, 2 * W + 4] = np.nan
    c[13, :] = np.nan
    tb, tc = torch.tensor(b, device=dev), torch.tensor(c, device=dev)
    out = K.rank_tests(tb, tc, pw_ref.PW_FRIEDMAN, 0.05, pods=(P, P), min_friedman=5)
    torch.cuda.synchronize()
    ref = pw_ref.rank_tests(torch.tensor(b, dtype=torch.float64), torch.tensor(c, dtype=torch.float64), pods=(P, P))
    fr = out["friedman"].cpu().double()
    np.testing.assert_array_equal(fr[:, 1].numpy(), ref.n_blocks.numpy())
    np.testing.assert_allclose(fr[:, 0].numpy(), ref.p_friedman.numpy(), rtol=2e-3, atol=1e-5)
    dref = pw_ref.pairwise_differs(ref, pw_ref.PW_FRIEDMAN, 0.05, min_friedman=5)
    assert (out["differs"].cpu().bool() == dref).float().mean() > 0.99
    assert 0 < int(dref.sum()) < N
    # the other tests are unchanged when Friedman rides along
    out2 = K.rank_tests(tb, tc, pw_ref.PW_ALL, 0.05, pods=(P, P), want_friedman=True)
    out3 = K.rank_tests(tb, tc, pw_ref.PW_ALL, 0.05)
    torch.cuda.synchronize()
    assert torch.equal(out2["pvals"], out3["pvals"]) and torch.equal(out2["differs"], out3["differs"])
    assert torch.equal(out2["friedman"], out["friedman"])


def test_bivariate_kernel(K):
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(4)
    N, T, C = 32, 2000, 6
    h = rng.multivariate_normal([1, 2], [[1.0, 0.6], [0.6, 2.0]], size=(N, T)).astype(np.float32)
    h[3, 10:20, 0] = np.nan
    hx = torch.tensor(h[..., 0], device=dev)
    hy = torch.tensor(h[..., 1], device=dev)
    cur = torch.tensor(rng.normal(1, 2, (N, C, 2)).astype(np.float32), device=dev)
    out = K.bivariate(hx, hy, 0, T, cur, torch.full((N,), 3.0, device=dev))
    torch.cuda.synchronize()
    fit = biv_ref.fit_bivariate(torch.tensor(h))
    d2 = biv_ref.mahalanobis2(fit, cur.cpu())
    np.testing.assert_allclose(out["d2"].cpu().numpy(), d2.numpy(), rtol=2e-3, atol=1e-3)
    assert torch.equal((d2 > 9.0).sum(1).int(), out["count"].cpu())


def test_ring_append(K):
    dev = torch.device("cuda:0")
    for dtype in (torch.float32, torch.bfloat16):
        dst = torch.zeros((10, 16), device=dev, dtype=dtype)
        src = torch.arange(50, dtype=torch.float32, device=dev).view(10, 5)
        K.ring_append(dst, 14, src)
        torch.cuda.synchronize()
        cols = [14, 15, 0, 1, 2]
        assert torch.equal(dst[:, cols].float(), src)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,m,T", [(torch.float32, 24, 24 * 9 + 5), (torch.bfloat16, 1440, 10080)])
def test_seasonal_decompose_kernel_matches_reference(K, dtype, m, T):
    from foremast_amd.models.decompose import seasonal_decompose as ref
    from foremast_amd.brain.engine import synthetic_history
    dev = torch.device("cuda:0")
    N, R = 64, T + 37
    y = synthetic_history(N, T, m, dev, seed=5)
    y[3, 100:140] = float("nan")
    ring = torch.full((N, R), float("nan"), device=dev, dtype=dtype)
    head = 29
    cols = (head + torch.arange(T, device=dev)) % R
    ring[:, cols] = y.to(dtype)
    out = K.seasonal_decompose(ring, head, T, m)
    torch.cuda.synchronize()
    d = ref(ring[:, cols].float().cpu(), m)
    scale = float(torch.nan_to_num(y.float()).abs().max())
    for k, r in (("trend", d.trend), ("seasonal", d.seasonal), ("resid", d.resid)):
        got = out[k].cpu()
        assert torch.equal(torch.isnan(got), torch.isnan(r)), k
        ok = ~torch.isnan(r)
        assert float((got[ok] - r[ok]).abs().max()) < 2e-4 * scale, k
    assert torch.allclose(out["phase_means"].cpu(), d.phase_means, atol=2e-4 * scale)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,m,T,aligned,head,split", [
    (torch.float32, 24, 24 * 9 + 5, False, 29, False), (torch.float32, 25, 25 * 6, False, 29, False),
    (torch.bfloat16, 1440, 10080, False, 29, False),
    # single-pass kernel (ring length a multiple of 8, m % 16 == 0): head phases, inline and
    # split (own-kernel) band / verdict, gapped series finished by the general kernel
    (torch.float32, 32, 32 * 9 + 5, True, 24, False), (torch.float32, 32, 32 * 9 + 5, True, 31, True),
    (torch.bfloat16, 1440, 10080, True, 29, False), (torch.bfloat16, 1440, 10080, True, 30, True),
    (torch.bfloat16, 1440, 10080, True, 35, True), (torch.float32, 1440, 10080, True, 32, True)])
def test_decompose_scorer_matches_reference(K, dtype, m, T, aligned, head, split):
    """ML_ALGORITHM=seasonal_decompose: K4's scoring mode (no [N, T] outputs) —
    trend extrapolation, phase means, residual RMS, band and verdicts — against
    models/decompose.py decompose_forecast + models/detect.py."""
    from foremast_amd.models import decompose as dec
    from foremast_amd.brain.engine import synthetic_history
    dev = torch.device("cuda:0")
    N, C = 64, 20
    R = (T + 40) // 8 * 8 if aligned else T + 37
    y = synthetic_history(N, T + C, m, dev, seed=6)
    y[3, 100:140] = float("nan")
    y[40, T - 1] = float("nan")
    ring = torch.full((N, R), float("nan"), device=dev, dtype=dtype)
    cols = (head + torch.arange(T, device=dev)) % R
    ring[:, cols] = y[:, :T].to(dtype)
    cur = y[:, T:].float().contiguous()
    cur[::5, 7] *= 1.5
    spec = _det_spec(K, N, C, dev, cur=cur, thr=3.0)
    if split:
        spec.max_horizon = C
    out = K.decompose_score(ring, head, T, m, spec)
    torch.cuda.synchronize()
    assert ("_sfc" in out) == split
    fc = dec.decompose_forecast(ring[:, cols].float().cpu(), m)
    scale = float(torch.nan_to_num(y.float()).abs().max())
    f_ref = dec.forecast_decomposition(fc, torch.arange(1, C + 1))
    assert float((out["forecast"].cpu() - f_ref).abs().max()) < 5e-4 * scale
    torch.testing.assert_close(out["sigma"].cpu(), fc.sigma, rtol=2e-3, atol=1e-4 * scale)
    assert torch.equal(out["nvalid"].cpu(), fc.n_valid)
    d = det_ref.detect(out["forecast"].cpu(), out["sigma"].cpu(), cur.cpu(), torch.full((N,), 3.0),
                       torch.full((N,), 3, dtype=torch.int8), torch.full((N,), -1e30))
    assert torch.equal(d.verdict, out["verdict"].cpu()) and torch.equal(d.count, out["count"].cpu())
    assert int((out["verdict"] == 1).sum()) >= N // 5 - 2
    if aligned and m % 16 == 0:  # the two gapped series took the general kernel (count reset after)
        assert int(out["_defer"][0]) == 0 and int(out["_defer"][-1]) == 0
        assert sorted(out["_defer"][1:3].tolist()) == [3, 40]


@pytest.mark.gpu
def test_decompose_scorer_many_deferred(K):
    """More gapped series than the deferred launch has workgroups (256): the
    grid-stride loop finishes every one of them, gap-free ones stay on the fast path."""
    from foremast_amd.models import decompose as dec
    from foremast_amd.brain.engine import synthetic_history
    dev = torch.device("cuda:0")
    N, m, T, C = 2600, 32, 32 * 9, 8
    y = synthetic_history(N, T + C, m, dev, seed=8)
    y[::2, 50] = float("nan")  # 1300 gapped series
    ring = y[:, :T].contiguous()
    cur = y[:, T:].contiguous()
    spec = _det_spec(K, N, C, dev, cur=cur, thr=3.0)
    spec.max_horizon = C
    out = K.decompose_score(ring, 0, T, m, spec)
    torch.cuda.synchronize()
    assert int(out["_defer"][0]) == 0
    assert sorted(out["_defer"][1:1 + N // 2].tolist()) == list(range(0, N, 2))
    fc = dec.decompose_forecast(ring.cpu(), m)
    scale = float(torch.nan_to_num(y).abs().max())
    f_ref = dec.forecast_decomposition(fc, torch.arange(1, C + 1))
    assert float((out["forecast"].cpu() - f_ref).abs().max()) < 5e-4 * scale
    torch.testing.assert_close(out["sigma"].cpu(), fc.sigma, rtol=2e-3, atol=1e-4 * scale)
    d = det_ref.detect(out["forecast"].cpu(), out["sigma"].cpu(), cur.cpu(), torch.full((N,), 3.0),
                       torch.full((N,), 3, dtype=torch.int8), torch.full((N,), -1e30))
    assert torch.equal(d.verdict, out["verdict"].cpu()) and torch.equal(d.count, out["count"].cpu())


@pytest.mark.gpu
@pytest.mark.parametrize("which", ["window_stats", "holt_winters"])
def test_anomaly_compaction_matches_band_flags(K, which):
    """K9: the compacted (series, col, value) list equals the points outside
    the enabled side of the band, computed on the host from the full bands."""
    from foremast_amd.brain.engine import synthetic_history
    dev = torch.device("cuda:0")
    N, T, m, C = 3000, 2 * 1440, 1440, 20
    hist = synthetic_history(N, T, m, dev, seed=11).to(torch.bfloat16)
    cur = hist[:, -C:].float().contiguous()
    cur[::7, 5] += 1000.0  # spikes
    cur[::11, 9] -= 1000.0
    bound = torch.tensor([1, 2, 3], dtype=torch.int8, device=dev).repeat(N // 3)
    spec = K.DetectSpec(horizons=torch.arange(1, C + 1, dtype=torch.int32, device=dev),
                        threshold=torch.full((N,), 3.0, device=dev), bound=bound,
                        min_lower=torch.full((N,), -1e9, device=dev), cur=cur,
                        anomalies=K.AnomalyBuffer(4096, dev))
    spec.anomalies.reset()
    if which == "window_stats":
        out = K.window_stats(hist, 0, T, spec)
    else:
        grid = sm_ref.make_grid(sm_ref.MODE_HW, (0.1, 0.5), (0.0, 0.1), (0.1, 0.5)).to(dev)
        out = K.smoothing_fit(hist, 0, T, sm_ref.MODE_HW, m, grid, spec)
    torch.cuda.synchronize()
    s, c, v, overflow = spec.anomalies.fetch()
    assert not overflow
    up, lo, x = out["upper"].cpu(), out["lower"].cpu(), cur.cpu()
    b = bound.cpu().long()[:, None]
    flag = (((b & 1) != 0) & (x > up)) | (((b & 2) != 0) & (x < lo))
    flag &= (out["verdict"].cpu()[:, None] >= 0)
    exp = flag.nonzero().numpy()
    assert len(exp) == len(s) and len(s) > 0
    assert (exp[:, 0] == s).all() and (exp[:, 1] == c).all()
    assert np.allclose(v, x.numpy()[s, c])
    assert (np.bincount(s, minlength=N) == out["count"].cpu().numpy()).all()


@pytest.mark.parametrize("variant", [4, 5])
@pytest.mark.parametrize("case", ["plain", "nan", "wrap_pad", "odd", "aligned_wrap_pad"])
def test_hw_half_variant_matches_reference(K, case, variant):
    """Variants 4/5 (two series per wave, 1440 = 32 x 45; 5 walks D = y - s over
    fp32 season differences): same fit as the fp64 reference and the same
    band/verdict semantics, on the flagship season."""
    dev = torch.device("cuda:0")
    m = 1440
    N = 17 if case == "odd" else 16
    T = 1440 * 4 + 300 if "wrap_pad" in case else 10080
    R, head = (T, 0)
    if case == "wrap_pad":
        R, head = T + 97, 61           # ring length not a multiple of 8: per-element staging
    elif case == "aligned_wrap_pad":
        R, head = T + 100, 1061        # multiple of 8, head mid-ring: 16-byte chunk staging
    if case == "plain":
        head = 3                       # aligned ring, head not a multiple of 8
    y = _series(N, T, m, seed=11 + len(case), nan_frac=0.01 if case == "nan" else 0.0)
    ring = torch.tensor(_ring(y, R, head), device=dev).to(torch.bfloat16)
    yl = ring.float().cpu().numpy()[:, (head + np.arange(T)) % R]
    grid = sm_ref.make_grid(sm_ref.MODE_HW, (0.1, 0.3, 0.5, 0.8), (0.0, 0.01, 0.05, 0.1), (0.05, 0.1, 0.3, 0.5))
    C = 50
    hz = torch.arange(1, 11, dtype=torch.int32).repeat(C // 10)
    cur = torch.tensor(y[:, -C:] * 1.05, device=dev)
    spec = K.DetectSpec(horizons=hz.to(dev), threshold=torch.full((N,), 2.0, device=dev),
                        bound=torch.full((N,), 3, dtype=torch.int8, device=dev),
                        min_lower=torch.full((N,), -1e30, device=dev), cur=cur, max_horizon=10)
    out = K.smoothing_fit(ring, head, T, sm_ref.MODE_HW, m, grid.to(dev), spec, variant=variant)
    torch.cuda.synchronize()
    assert K.last_hw_variant == variant
    ref = sm_ref.fit_smoothing(torch.tensor(yl, dtype=torch.float64), sm_ref.MODE_HW, grid.double(), m=m)
    kb = out["best"].cpu().long()
    same = (kb == ref.best).numpy()
    assert same.mean() >= 0.75
    _assert_near_optimal(yl, grid, sm_ref.MODE_HW, m, kb)
    np.testing.assert_allclose(out["sigma"].cpu().numpy(), ref.sigma.numpy(), rtol=5e-3)
    np.testing.assert_allclose(out["level"].cpu().numpy()[same], ref.level.numpy()[same], rtol=2e-3, atol=5e-3)
    f_ref = sm_ref.forecast(ref, hz.long())
    np.testing.assert_allclose(out["forecast"].cpu().numpy()[same], f_ref.numpy()[same], rtol=5e-3, atol=2e-2)
    d = _ref_detect(out, grid, sm_ref.MODE_HW, m, hz, cur)
    assert torch.equal(d.count, out["count"].cpu())
    assert torch.equal(d.verdict, out["verdict"].cpu())
    # variant 3 (one series per wave) on the same input agrees on the chosen grid point
    out3 = K.smoothing_fit(ring, head, T, sm_ref.MODE_HW, m, grid.to(dev), spec, variant=3)
    torch.cuda.synchronize()
    assert (out3["best"].cpu() == out["best"].cpu()).float().mean() >= 0.9


@pytest.mark.parametrize("N", [40, 1030])
def test_hw_split_tail_matches_whole_pairs(K, N, monkeypatch):
    """Variant 5's split tail (the grid of a series pair fitted by two workgroups,
    merged by the second arriver through device-scope sc1 stores / loads) gives
    exactly the whole-pair result."""
    dev = torch.device("cuda:0")
    m, T = 1440, 4320
    y = _series(N, T, m, seed=21, nan_frac=0.0)
    y[3, 2000] = np.nan  # one gapped pair goes to the general kernel in both runs
    ring = torch.tensor(y, device=dev).to(torch.bfloat16)
    grid = sm_ref.make_grid(sm_ref.MODE_HW, (0.1, 0.3, 0.5, 0.8), (0.0, 0.01, 0.05, 0.1), (0.05, 0.1, 0.3, 0.5))
    hz = torch.arange(1, 11, dtype=torch.int32).repeat(2)
    cur = torch.tensor(y[:, -20:] * 1.04, device=dev)
    spec = K.DetectSpec(horizons=hz.to(dev), threshold=torch.full((N,), 2.0, device=dev),
                        bound=torch.full((N,), 3, dtype=torch.int8, device=dev),
                        min_lower=torch.full((N,), -1e30, device=dev), cur=cur, max_horizon=10)
    lib = K.nat.require()
    slots = K._split_workspace(dev)[1]
    S = lib.fm_hw_d_split_plan((N + 1) // 2, slots, K.SPLIT_MAX)
    assert S > 0
    outs = []
    for split in ("1", "0"):
        monkeypatch.setenv("FOREMAST_HW_SPLIT", split)
        outs.append({k: v.clone() for k, v in
                     K.smoothing_fit(ring, 0, T, sm_ref.MODE_HW, m, grid.to(dev), spec, variant=5).items()})
        torch.cuda.synchronize()
    for key in ("best", "level", "trend", "sigma", "verdict", "count", "forecast", "upper", "lower"):
        assert torch.equal(outs[0][key], outs[1][key]), key


@pytest.mark.parametrize("N,split", [(64, "0"), (1030, "1"), (4096, "0")])
def test_hw_grid_pruning_is_exact(K, N, split, monkeypatch):
    """Variant 5's grid branch and bound (a wave drops a grid pair once its partial SSE
    exceeds the best complete SSE of the block) returns exactly the exhaustive fit:
    every output bit for bit, on series whose grid SSEs are close (low noise), spread
    (level shifts, spikes) and tied (constant series)."""
    dev = torch.device("cuda:0")
    m, T = 1440, 10080
    y = _series(N, T, m, seed=31, nan_frac=0.0)
    rng = np.random.default_rng(5)
    y[1::7] += rng.normal(0.0, 5.0, size=y[1::7].shape)            # noisy: every pair close
    y[2::7, 6000:] += 40.0                                          # level shift: alpha matters
    y[3::7, rng.integers(1440, T, 50)] += 300.0                     # spikes
    y[4::7] = 7.0                                                   # constant: every SSE ties at 0
    y[5::7] *= np.linspace(1.0, 3.0, T)                             # growing amplitude
    ring = torch.tensor(y, device=dev).to(torch.bfloat16)
    grid = sm_ref.make_grid(sm_ref.MODE_HW, (0.1, 0.3, 0.5, 0.8), (0.0, 0.01, 0.05, 0.1), (0.05, 0.1, 0.3, 0.5))
    hz = torch.arange(1, 11, dtype=torch.int32).repeat(5)
    cur = torch.tensor(y[:, -50:] * 1.04, device=dev)
    spec = K.DetectSpec(horizons=hz.to(dev), threshold=torch.full((N,), 2.0, device=dev),
                        bound=torch.full((N,), 3, dtype=torch.int8, device=dev),
                        min_lower=torch.full((N,), -1e30, device=dev), cur=cur, max_horizon=10)
    monkeypatch.setenv("FOREMAST_HW_SPLIT", split)

    def fit(prune, out=None):
        monkeypatch.setenv("FOREMAST_HW_PRUNE", prune)
        o = K.smoothing_fit(ring, 0, T, sm_ref.MODE_HW, m, grid.to(dev), spec, variant=5, out=out)
        torch.cuda.synchronize()
        return o

    ref = {k: v.clone() for k, v in fit("0").items()}
    reused = fit("1")                                      # out["best"] is uninitialised: arbitrary hints
    runs = [{k: v.clone() for k, v in reused.items()}]
    runs.append({k: v.clone() for k, v in fit("1", reused).items()})  # hints = the previous winners
    reused["best"].copy_(torch.randint(-3, 70, (N,), dtype=torch.int32, device=dev))  # wrong / out-of-range hints
    runs.append({k: v.clone() for k, v in fit("1", reused).items()})
    for o in runs:
        for key in ("best", "level", "trend", "sigma", "verdict", "count", "forecast", "upper", "lower"):
            assert torch.equal(o[key], ref[key]), key


def test_hw_split_plan():
    from foremast_amd.ops import _native as nat
    lib = nat.require()
    assert lib.fm_hw_d_split_plan(6250, 512, 4096) == 106   # 12.5k series/GPU: split the last partial round
    assert lib.fm_hw_d_split_plan(50000, 512, 4096) == 0    # 100k: the tail is already negligible
    assert lib.fm_hw_d_split_plan(20, 512, 4096) == 20      # tiny batches: every pair in two halves
    assert lib.fm_hw_d_split_plan(20, 0, 4096) == 0


@pytest.mark.parametrize("shift,one_step", [(0.0, False), (1.0, False), (1.0, True)])
@pytest.mark.parametrize("which", ["window_stats", "holt_winters", "hw_deferred"])
def test_two_rule_detection_matches_reference(K, which, shift, one_step):
    """Full band + lowered pairwise band that needs >= pw_min_points points, and
    (shift > 0) the mean-shift rule (detect.h det_decide): kernel verdicts, counts,
    bands and the K9 list equal the reference on series built to sit on each side
    of every rule.  one_step: the rule's spread is the one-step sigma (DetectSpec
    shift_one_step / detect's shift_sigma), not the horizon-scaled band sigma."""
    from foremast_amd.brain.engine import synthetic_history
    dev = torch.device("cuda:0")
    N, T, m, C = 2000, 2 * 1440, 1440, 10
    hist = synthetic_history(N, T, m, dev, seed=5).to(torch.bfloat16)
    g = torch.Generator(device=dev).manual_seed(3)
    hf = hist.float()
    # noise on the scale of each model's sigma, so both rules fire on some series and not others
    scale = hf.std(1, keepdim=True) if which == "window_stats" else (hf[:, 1:] - hf[:, :-1]).std(1, keepdim=True)
    cur = (hf[:, -C:] + torch.randn((N, C), generator=g, device=dev) * scale).contiguous()
    if shift:  # sustained level shifts around the mean-shift threshold on a quarter of the series
        sgn = torch.where(torch.arange(N, device=dev) % 16 < 8, 1.0, -1.0)[:, None]
        lift = (torch.arange(N, device=dev) % 8 >= 6).float()[:, None]
        cur = (cur + lift * sgn * 1.3 * shift * scale).contiguous()
    differs = (torch.arange(N, device=dev) % 2).to(torch.uint8)
    # baseline pods: on the history's level (+ noise), none for every 32nd series
    bmean = (hf[:, -C:].mean(1) + torch.randn((N,), generator=g, device=dev) * scale[:, 0] * 0.2).contiguous()
    bmean[::32] = float("nan")
    thr = torch.full((N,), 3.0, device=dev)
    bound = torch.tensor([1, 2, 3, 3], dtype=torch.int8, device=dev).repeat(N // 4)
    full, low = det_ref.effective_thresholds(thr.cpu(), bound.cpu(), C, 0.5, "sidak")
    spec = K.DetectSpec(horizons=torch.arange(1, C + 1, dtype=torch.int32, device=dev), threshold=full.to(dev),
                        bound=bound, min_lower=torch.full((N,), -1e9, device=dev), cur=cur, differs=differs,
                        threshold_low=low.to(dev), pw_min_points=3, anomalies=K.AnomalyBuffer(N * C, dev),
                        max_horizon=C, shift_threshold=shift, base_mean=bmean, shift_min_points=5,
                        shift_one_step=one_step)
    spec.anomalies.reset()
    grid = sm_ref.make_grid(sm_ref.MODE_HW, (0.1, 0.5), (0.0, 0.1), (0.1, 0.5)).to(dev)
    if which == "window_stats":
        out = K.window_stats(hist, 0, T, spec)
        sig = out["std"].cpu()
        sig1 = sig
    else:
        if which == "hw_deferred":
            out = K.smoothing_fit(hist, 0, T, sm_ref.MODE_HW, m, grid, spec, defer_detect=True, variant=5)
            if K.last_detect_deferred:
                Tp = K.smoothing_geometry(sm_ref.MODE_HW, T, m)[0]
                K.hw_detect_deferred(out, spec, Tp, m, grid=grid)
        else:
            out = K.smoothing_fit(hist, 0, T, sm_ref.MODE_HW, m, grid, spec)
        params = grid.cpu()[out["best"].cpu().long()]
        sig1 = out["sigma"].cpu()
        sig = sig1[:, None] * det_ref.horizon_sigma_factor(params, sm_ref.MODE_HW, m, torch.arange(1, C + 1))
    torch.cuda.synchronize()
    d = det_ref.detect(out["forecast"].cpu(), sig, cur.cpu(), full, bound.cpu(), torch.full((N,), -1e9),
                       differs=differs.cpu(), threshold_low=low, pw_min_points=3, shift_threshold=shift,
                       base_mean=bmean.cpu(), shift_min_points=5, shift_sigma=sig1 if one_step else None)
    assert torch.equal(d.verdict, out["verdict"].cpu())
    assert torch.equal(d.count, out["count"].cpu())
    low_fired = (differs.cpu().bool() & (d.count > 0))
    assert int(low_fired.sum()) > 0 and int((d.verdict == 0).sum()) > 0  # both sides exercised
    if shift:
        d0 = det_ref.detect(out["forecast"].cpu(), sig, cur.cpu(), full, bound.cpu(), torch.full((N,), -1e9),
                            differs=differs.cpu(), threshold_low=low, pw_min_points=3)
        by_shift = (d.verdict == 1) & (d0.verdict == 0)
        assert int(by_shift.sum()) > 0 and not bool((by_shift & ~differs.cpu().bool()).any())
    np.testing.assert_allclose(out["upper"].cpu().numpy(), d.upper.numpy(), rtol=1e-4, atol=1e-3)
    s_, c_, v_, overflow = spec.anomalies.fetch()
    assert not overflow
    exp = d.anomaly.nonzero().numpy()
    assert len(exp) == len(s_) and (exp[:, 0] == s_).all() and (exp[:, 1] == c_).all()
