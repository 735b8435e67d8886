"""Oracle tests for the reference scorers: scipy for the rank tests, a
textbook (non error-correction) numpy Holt-Winters for the smoothing family."""

import math

import numpy as np
import pytest
import scipy.stats as ss
import torch

from foremast_amd.models import bivariate, detect, moving_average, pairwise, smoothing


def _textbook_hw(y, m, a, b, g, mode):
    """Textbook additive Holt-Winters one-step SSE (numpy, float64)."""
    y = np.asarray(y, dtype=np.float64)
    T = len(y)
    if mode == smoothing.MODE_HW:
        Tp = ((T + m - 1) // m) * m
        y = np.concatenate([np.full(Tp - T, np.nan), y])
        l = np.nanmean(y[:m])
        bb = (np.nanmean(y[m:2 * m]) - l) / m
        s = np.where(np.isnan(y[:m]), 0.0, y[:m] - l)
        t0 = m
    else:
        Tp = T
        first = np.argmax(~np.isnan(y))
        l = y[first]
        bb = 0.0
        s = np.zeros(1)
        m = 1
        t0 = 0
    sse = 0.0
    n = 0
    for t in range(t0, Tp):
        p = t % m
        sp = s[p] if mode == smoothing.MODE_HW else 0.0
        yhat = l + bb + sp
        yt = y[t]
        if np.isnan(yt):
            yt = yhat
        else:
            sse += (yt - yhat) ** 2
            n += 1
        ln = a * (yt - sp) + (1 - a) * (l + bb)
        bn = b * (ln - l) + (1 - b) * bb
        if mode == smoothing.MODE_HW:
            s[p] = g * (yt - ln) + (1 - g) * sp
        l, bb = ln, bn
    return sse, n, l, bb, s, Tp


@pytest.mark.parametrize("mode", [smoothing.MODE_ES, smoothing.MODE_DES, smoothing.MODE_HW])
def test_smoothing_matches_textbook(mode):
    rng = np.random.default_rng(0)
    m = 12
    N, T = 5, 5 * m + 7
    t = np.arange(T)
    y = (10 + 0.05 * t + 3 * np.sin(2 * np.pi * t / m))[None, :] + rng.normal(0, 0.5, (N, T))
    y[1, 5] = np.nan
    y[2, 30:33] = np.nan
    grid = smoothing.make_grid(mode, (0.2, 0.6), (0.0, 0.1), (0.1, 0.4))
    fit = smoothing.fit_smoothing(torch.tensor(y, dtype=torch.float32), mode, grid, m=m)
    for i in range(N):
        best = None
        for gi, (a, b, g) in enumerate(grid.tolist()):
            sse, n, l, bb, s, Tp = _textbook_hw(y[i], m, a, b, g, mode)
            if best is None or sse < best[0]:
                best = (sse, n, l, bb, s, gi, Tp)
        sse, n, l, bb, s, gi, Tp = best
        assert int(fit.best[i]) == gi
        assert fit.sigma[i].item() == pytest.approx(math.sqrt(sse / n), rel=1e-4)
        assert fit.level[i].item() == pytest.approx(l, rel=1e-4, abs=1e-4)
        assert fit.trend[i].item() == pytest.approx(bb, rel=1e-3, abs=1e-4)
        h = torch.tensor([1, 2, 5])
        f = smoothing.forecast(fit, h)[i].numpy()
        sp = [s[(Tp - 1 + k) % len(s)] if mode == smoothing.MODE_HW else 0.0 for k in (1, 2, 5)]
        exp = [l + k * bb + sp[j] for j, k in enumerate((1, 2, 5))]
        np.testing.assert_allclose(f, exp, rtol=1e-4, atol=1e-3)


def test_rank_tests_vs_scipy():
    rng = np.random.default_rng(1)
    N, nb, nc = 12, 30, 25
    b = rng.normal(0, 1, (N, nb))
    c = rng.normal(0.3, 1, (N, nc))
    # ties and a NaN-padded row
    b[0] = np.round(b[0], 0)
    c[0] = np.round(c[0], 0)
    b[3, 20:] = np.nan
    c[4, :5] = np.round(b[4, :5], 1)
    b[4, :5] = np.round(b[4, :5], 1)
    res = pairwise.rank_tests(torch.tensor(b, dtype=torch.float64), torch.tensor(c, dtype=torch.float64))
    for i in range(N):
        bi = b[i][~np.isnan(b[i])]
        ci = c[i][~np.isnan(c[i])]
        mw = ss.mannwhitneyu(bi, ci, alternative="two-sided", use_continuity=True, method="asymptotic")
        assert res.p_mw[i].item() == pytest.approx(mw.pvalue, rel=1e-4, abs=1e-6)
        kw = ss.kruskal(bi, ci)
        assert res.p_kruskal[i].item() == pytest.approx(kw.pvalue, rel=1e-4, abs=1e-6)
        k = min(nb, nc)
        d = c[i, :k] - b[i, :k]
        ok = ~np.isnan(d)
        bw, cw = b[i, :k][ok], c[i, :k][ok]
        w = ss.wilcoxon(cw, bw, zero_method="wilcox", correction=False, method="approx")
        assert res.p_wilcoxon[i].item() == pytest.approx(w.pvalue, rel=1e-4, abs=1e-6)


def test_friedman_vs_scipy():
    rng = np.random.default_rng(2)
    g = rng.normal(0, 1, (3, 10, 4))
    g[1] = np.round(g[1])
    p = pairwise.friedman(torch.tensor(g, dtype=torch.float64))
    for i in range(3):
        exp = ss.friedmanchisquare(*[g[i, :, j] for j in range(4)]).pvalue
        assert p[i].item() == pytest.approx(exp, rel=1e-4)


def test_friedman_pods_vs_scipy():
    """Time slots x pods (2 baseline + 2 canary pods): scipy's friedmanchisquare
    over the blocks valid in every pod."""
    rng = np.random.default_rng(5)
    N, Pb, Pc, W = 6, 2, 2, 12
    b = rng.normal(0, 1, (N, Pb * W))
    c = rng.normal(0.4, 1, (N, Pc * W))
    b[1] = np.round(b[1])
    c[1] = np.round(c[1])
    b[2, 3] = np.nan      # slot 3 incomplete in series 2
    c[3, W + 5] = np.nan  # slot 5 of canary pod 1 in series 3
    p, nblk = pairwise.friedman_pods(torch.tensor(b), torch.tensor(c), Pb, Pc)
    for i in range(N):
        g = np.concatenate([b[i].reshape(Pb, W), c[i].reshape(Pc, W)], 0)  # [k, W]
        ok = ~np.isnan(g).any(0)
        exp = ss.friedmanchisquare(*[g[t, ok] for t in range(Pb + Pc)]).pvalue
        assert int(nblk[i]) == int(ok.sum())
        assert p[i].item() == pytest.approx(exp, rel=1e-5)
    res = pairwise.rank_tests(torch.tensor(b), torch.tensor(c), pods=(Pb, Pc))
    d = pairwise.pairwise_differs(res, pairwise.PW_FRIEDMAN, 0.05, min_friedman=5)
    assert d.tolist() == ((p < 0.05) & (nblk >= 5)).tolist()
    assert pairwise.PW_BY_NAME["FRIEDMAN"] == pairwise.PW_FRIEDMAN


def test_pairwise_decision_modes():
    N = 4
    r = pairwise.PairwiseResult(
        p_mw=torch.tensor([0.01, 0.01, 0.5, 0.01]), p_wilcoxon=torch.tensor([0.01, 0.5, 0.5, 0.01]),
        p_kruskal=torch.tensor([0.01, 0.01, 0.5, 0.01]), n_base=torch.tensor([30., 30., 30., 3.]),
        n_cur=torch.tensor([30., 30., 30., 3.]), n_pairs=torch.tensor([30., 30., 30., 3.]))
    assert pairwise.pairwise_differs(r, pairwise.PW_ALL, 0.05).tolist() == [True, False, False, False]
    assert pairwise.pairwise_differs(r, pairwise.PW_ANY, 0.05).tolist() == [True, True, False, False]
    assert pairwise.pairwise_differs(r, pairwise.PW_MANN_WHITE, 0.05).tolist() == [True, True, False, False]


def test_window_stats_and_detect():
    rng = np.random.default_rng(3)
    y = rng.normal(5, 2, (6, 200)).astype(np.float32)
    y[2, :50] = np.nan
    st = moving_average.window_stats(torch.tensor(y))
    np.testing.assert_allclose(st.mean.numpy(), np.nanmean(y, 1), rtol=1e-5)
    np.testing.assert_allclose(st.std.numpy(), np.nanstd(y, 1), rtol=1e-4)
    stw = moving_average.window_stats(torch.tensor(y), window=60)
    np.testing.assert_allclose(stw.mean.numpy(), np.nanmean(y[:, -60:], 1), rtol=1e-5)
    f = st.mean[:, None].expand(6, 4)
    x = torch.tensor(np.array([[5, 5, 5, 100]] * 6, dtype=np.float32))
    x[5] = float("nan")
    d = detect.detect(f, st.std, x, torch.full((6,), 2.0), torch.tensor([1, 2, 3, 1, 1, 1]),
                      torch.zeros(6))
    assert d.verdict.tolist() == [1, 0, 1, 1, 1, -1]


def test_bivariate():
    rng = np.random.default_rng(4)
    cov = np.array([[1.0, 0.6], [0.6, 2.0]])
    h = rng.multivariate_normal([1, 2], cov, size=(3, 4000))
    fit = bivariate.fit_bivariate(torch.tensor(h))
    x = torch.tensor([[[1.0, 2.0], [4.0, -1.0]]] * 3)
    d2 = bivariate.mahalanobis2(fit, x)
    inv = np.linalg.inv(np.cov(h[0].T, bias=True))
    dv = np.array([3.0, -3.0]) - (h[0].mean(0) - np.array([1, 2]))
    exp = dv @ inv @ dv
    assert d2[0, 1].item() == pytest.approx(exp, rel=1e-3)
    assert d2[0, 0].item() < 0.1


def test_prophet_lite_recovers_trend_and_seasonality():
    """Parity unpinned (the prophet package is not installed): checks the
    batched ridge fit against the generating model, gap handling, and that a
    batch equals independent per-series fits."""
    import math
    from foremast_amd.models import prophet_lite as P
    torch.manual_seed(0)
    B, T, step = 3, 3 * 1440, 60.0
    end = torch.full((B,), 1.7e9, dtype=torch.float64)
    j = torch.arange(T, dtype=torch.float64)
    ts = end[:, None] - (T - 1 - j) * step

    def truth(t):
        return 20 + 4 * torch.sin(2 * math.pi * t / 86400 + torch.arange(B)[:, None]) + 2e-5 * (t - 1.69e9)
    y = truth(ts) + 0.2 * torch.randn(B, T, dtype=torch.float64)
    y[1, 500:900] = float("nan")
    fit = P.fit_prophet(y.float(), end, torch.full((B,), step))
    assert fit.seasons and fit.seasons[0][0] == P.DAY
    assert torch.allclose(fit.sigma, torch.full((B,), 0.2), atol=0.03)
    cts = end[:, None] + torch.arange(1, 31, dtype=torch.float64)[None, :] * step
    f = P.forecast(fit, cts)
    assert float((f - truth(cts)).abs().max()) < 0.15
    one = P.fit_prophet(y[1:2].float(), end[1:2], torch.full((1,), step))
    assert torch.allclose(P.forecast(one, cts[1:2]), f[1:2], atol=1e-4)


def test_seasonal_decompose_reference():
    import math
    from foremast_amd.models.decompose import seasonal_decompose
    torch.manual_seed(1)
    N, m, P = 3, 24, 8
    T = m * P
    t = torch.arange(T, dtype=torch.float64)
    season = torch.sin(2 * math.pi * t / m)
    y = 5 + 0.01 * t + 2 * season + 0.01 * torch.randn(N, T, dtype=torch.float64)
    d = seasonal_decompose(y, m)
    h = m // 2
    assert torch.isnan(d.trend[:, :h]).all() and torch.isnan(d.trend[:, T - h:]).all()
    mid = slice(h, T - h)
    assert torch.allclose(d.trend[:, mid], (5 + 0.01 * t[mid]).expand(N, -1), atol=0.02)
    assert torch.allclose(d.seasonal, 2 * season.expand(N, -1), atol=0.03)
    assert abs(float(d.phase_means.sum(1).abs().max())) < 1e-9
    assert float(d.resid[:, mid].abs().max()) < 0.06
    # gaps: still defined where at least half of the window is valid
    y2 = y.clone()
    y2[:, 50:55] = float("nan")
    d2 = seasonal_decompose(y2, m)
    assert torch.isfinite(d2.trend[:, 52]).all() and torch.allclose(d2.seasonal, d.seasonal, atol=0.05)


def test_horizon_sigma_factor_matches_direct_sum():
    """Closed form of the h-step forecast-error factor equals the direct sum of
    c_j^2 (c_j = a (1 + j b) + g (1 - a) [j mod m == 0]) for ES / DES / HW."""
    rng = np.random.default_rng(7)
    params = torch.tensor(rng.uniform(0.05, 0.9, (5, 3)), dtype=torch.float32)
    h = torch.arange(1, 40)
    for mode, m in ((0, 0), (1, 0), (2, 7), (2, 1)):
        got = detect.horizon_sigma_factor(params, mode, m, h).double().numpy()
        for i in range(5):
            a, b, g = params[i].double().tolist()
            b = b if mode >= 1 else 0.0
            for k, hh in enumerate(h.tolist()):
                v = 1.0
                for j in range(1, hh):
                    c = a * (1 + j * b) + (g * (1 - a) if mode == 2 and m > 0 and j % m == 0 else 0.0)
                    v += c * c
                assert got[i, k] == pytest.approx(np.sqrt(v), rel=1e-5)


def test_window_threshold_sidak():
    """P(any of C points outside the corrected band) equals P(one point outside
    the uncorrected band), on the sides the bound enables."""
    from scipy import stats
    thr = torch.tensor([2.0, 3.0, 4.0, 2.0])
    bound = torch.tensor([1, 2, 3, 3], dtype=torch.int8)
    for C in (1, 10, 50):
        z = detect.window_threshold(thr, bound, C).double().numpy()
        for i in range(4):
            sides = 2 if int(bound[i]) == 3 else 1
            p1 = sides * stats.norm.sf(float(thr[i]))
            pc = sides * stats.norm.sf(z[i])
            assert 1 - (1 - pc) ** C == pytest.approx(p1, rel=1e-4)
    assert torch.equal(detect.window_threshold(thr, bound, 50, "none"), thr)


def test_pairwise_lowered_band_needs_min_points():
    """The lowered band applies only when differs AND >= pw_min_points points
    fall outside it; one point outside the full band always flags."""
    f = torch.zeros(4, 10)
    sig = torch.ones(4)
    x = torch.zeros(4, 10)
    x[0, :2] = 2.5      # 2 points between the lowered (2) and full (4) bands
    x[1, :3] = 2.5      # 3 such points
    x[2, 0] = 5.0       # one spike beyond the full band
    x[3, :3] = 2.5      # 3 points, but baseline and current do not differ
    thr = torch.full((4,), 4.0)
    low = torch.full((4,), 2.0)
    differs = torch.tensor([1, 1, 0, 0], dtype=torch.uint8)
    d = detect.detect(f, sig, x, thr, torch.full((4,), 3, dtype=torch.int8), torch.full((4,), -1e9),
                      differs=differs, threshold_low=low, pw_min_points=3)
    assert d.verdict.tolist() == [0, 1, 1, 0]
    assert d.count.tolist() == [0, 3, 1, 0]
    assert float(d.upper[1, 0]) == 2.0 and float(d.upper[0, 0]) == 4.0  # band of the rule in force
    d1 = detect.detect(f, sig, x, thr, torch.full((4,), 3, dtype=torch.int8), torch.full((4,), -1e9),
                       differs=differs, threshold_low=low, pw_min_points=1)
    assert d1.verdict.tolist() == [1, 1, 1, 0]


def test_pairwise_mean_shift_rule():
    """With differs and no band fired, a canary window whose mean deviation from the
    baseline pods' mean is beyond shift_threshold sigmas (on a side bound enables) is
    anomalous; its band is base_mean +- shift * s and its count the points outside it.
    A forecast error does not trigger it: only the distance to the baseline counts."""
    f = torch.zeros(6, 10)
    sig = torch.ones(6)
    x = torch.full((6, 10), 1.6)    # every point 1.6 sigma above the baseline: inside both bands
    x[1] = -1.6                      # down, upper-only bound below
    x[2, :5] = 0.0                   # mean 0.8: below the shift threshold
    x[4, 0] = float("nan")           # missing points do not count
    bm = torch.zeros(6)
    bm[5] = 1.6                      # canary on its baseline, 1.6 sigma off the forecast: healthy
    thr, low = torch.full((6,), 4.0), torch.full((6,), 2.0)
    bound = torch.tensor([3, 1, 3, 3, 2, 3], dtype=torch.int8)
    differs = torch.tensor([1, 1, 1, 0, 1, 1], dtype=torch.uint8)
    kw = dict(differs=differs, threshold_low=low, pw_min_points=3, shift_min_points=9)
    d0 = detect.detect(f, sig, x, thr, bound, torch.full((6,), -1e9), **kw)
    assert d0.verdict.tolist() == [0] * 6
    d = detect.detect(f, sig, x, thr, bound, torch.full((6,), -1e9), shift_threshold=1.5, base_mean=bm, **kw)
    assert d.verdict.tolist() == [1, 0, 0, 0, 0, 0]  # row 4: upward shift, lower-only bound
    assert d.count.tolist() == [10, 0, 0, 0, 0, 0]
    assert float(d.upper[0, 0]) == 1.5 and float(d.upper[2, 0]) == 4.0
    x[4] = -1.6
    x[4, 0] = float("nan")
    d = detect.detect(f, sig, x, thr, bound, torch.full((6,), -1e9), shift_threshold=1.5, base_mean=bm, **kw)
    assert d.verdict.tolist() == [1, 0, 0, 0, 1, 0] and d.count.tolist()[4] == 9
    d = detect.detect(f, sig, x, thr, bound, torch.full((6,), -1e9), shift_threshold=1.5, base_mean=bm,
                      **{**kw, "shift_min_points": 10})
    assert d.verdict.tolist() == [1, 0, 0, 0, 0, 0]  # row 4 has 9 valid points: too few
    bm[0] = float("nan")             # no baseline values: no mean-shift rule
    d = detect.detect(f, sig, x, thr, bound, torch.full((6,), -1e9), shift_threshold=1.5, base_mean=bm, **kw)
    assert d.verdict.tolist()[0] == 0


def test_mean_shift_rule_one_step_spread():
    """shift_sigma: the mean-shift rule measures the window against the baseline in units of
    the one-step sigma, while the bands keep the horizon-scaled sigma.  A +2 sigma shift whose
    band sigma grows to 1.5x over the window: under the horizon-scaled spread the window's mean
    z is ~1.3 (below 1.5, healthy); in one-step units it is 2.0 (anomalous)."""
    N, C = 2, 10
    f = torch.zeros(N, C)
    sig1 = torch.ones(N)
    sig = sig1[:, None] * torch.linspace(1.0, 2.0, C)[None, :]     # horizon-scaled (mean 1.5)
    x = torch.full((N, C), 2.0)
    x[1] = 0.5                                                     # a small shift stays healthy
    thr, low = torch.full((N,), 4.0), torch.full((N,), 3.0)
    bound = torch.full((N,), 3, dtype=torch.int8)
    kw = dict(differs=torch.ones(N, dtype=torch.uint8), threshold_low=low, pw_min_points=3, shift_min_points=5,
              shift_threshold=1.5, base_mean=torch.zeros(N))
    d_h = detect.detect(f, sig, x, thr, bound, torch.full((N,), -1e9), **kw)
    d_1 = detect.detect(f, sig, x, thr, bound, torch.full((N,), -1e9), shift_sigma=sig1, **kw)
    assert d_h.verdict.tolist() == [0, 0] and d_1.verdict.tolist() == [1, 0]
    assert d_1.count.tolist() == [10, 0]
    np.testing.assert_allclose(d_1.upper[0].numpy(), 1.5)           # band base_mean + 1.5 * one-step sigma
    np.testing.assert_allclose(d_1.upper[1].numpy(), (4.0 * sig[1]).numpy())  # others keep the scaled band


def test_decompose_forecast_continues_trend_and_season():
    """Decomposition scorer reference: on a noiseless linear trend + sinusoid the
    forecast matches the generating function and the residual RMS is ~0."""
    import math
    from foremast_amd.models import decompose as dec
    m, T = 24, 24 * 6
    t = torch.arange(T + 10, dtype=torch.float64)
    y = (5.0 + 0.01 * t + torch.sin(2 * math.pi * t / m)).float()[None].repeat(3, 1)
    fc = dec.decompose_forecast(y[:, :T], m)
    f = dec.forecast_decomposition(fc, torch.arange(1, 11))
    torch.testing.assert_close(f, y[:, T:], rtol=0, atol=2e-3)
    assert float(fc.sigma.max()) < 1e-3 and int(fc.n_valid[0]) == T


def test_decompose_sigma_is_a_prediction_spread():
    """The decomposition scorer's sigma predicts the spread of NEW points: on a
    trend + season + unit noise, the RMS of (next-day value - forecast) matches
    sigma (the in-sample residual RMS alone is ~15 % too small at K = 6 seasons)."""
    import math
    from foremast_amd.models import decompose as dec
    g = torch.Generator().manual_seed(5)
    N, m, K = 400, 48, 7
    T = m * K
    H = 10
    t = torch.arange(T + H, dtype=torch.float64)
    phase = torch.rand(N, 1, generator=g, dtype=torch.float64) * 2 * math.pi
    clean = 10.0 + 0.002 * t + 3.0 * torch.sin(2 * math.pi * t / m + phase)
    y = (clean + torch.randn(N, T + H, generator=g, dtype=torch.float64)).float()
    fc = dec.decompose_forecast(y[:, :T], m)
    f = dec.forecast_decomposition(fc, torch.arange(1, H + 1))
    err_rms = float(((y[:, T:] - f) ** 2).mean().sqrt())
    sig = float(fc.sigma.mean())
    assert abs(sig / err_rms - 1.0) < 0.08, (sig, err_rms)
    raw = sig / dec.prediction_factor(T, m)  # the plain in-sample residual RMS
    assert raw / err_rms < 0.92
