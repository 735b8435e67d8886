"""Property-based tests: ties, constant series, NaNs and
short windows for the scorers against scipy/numpy oracles; round-trips for
the wire codecs."""

import math

import numpy as np
import pytest
import scipy.stats as ss
import torch
from hypothesis import HealthCheck, assume, given, settings
from hypothesis import strategies as st

from foremast_amd.api import crd
from foremast_amd.api.gojson import from_go, to_go
from foremast_amd.models import decompose, detect, moving_average, pairwise
from foremast_amd.promql.selector import parse_selector
from foremast_amd.service import urls

SETTINGS = settings(max_examples=60, deadline=None, suppress_health_check=[HealthCheck.too_slow])

vals = st.floats(min_value=-50, max_value=50, allow_nan=False, width=32)


def _sample(draw, n_lo, n_hi, ties):
    n = draw(st.integers(n_lo, n_hi))
    xs = draw(st.lists(vals, min_size=n, max_size=n))
    if ties:
        xs = [round(v) for v in xs]  # many ties
    return np.array(xs, dtype=np.float64)


@st.composite
def two_samples(draw):
    ties = draw(st.booleans())
    return _sample(draw, 3, 40, ties), _sample(draw, 3, 40, ties)


@SETTINGS
@given(two_samples())
def test_mann_whitney_and_kruskal_match_scipy(bc):
    b, c = bc
    assume(len(np.unique(np.concatenate([b, c]))) > 1)  # scipy is undefined when all values tie
    nb, nc = len(b), len(c)
    B = np.full((1, 40), np.nan)
    C = np.full((1, 40), np.nan)
    B[0, :nb] = b
    C[0, :nc] = c
    res = pairwise.rank_tests(torch.tensor(B), torch.tensor(C))
    mw = ss.mannwhitneyu(b, c, alternative="two-sided", use_continuity=True, method="asymptotic")
    kw = ss.kruskal(b, c)
    # fp32 statistics (as in the kernel): near p = 1 the chi2/normal tail is
    # sqrt-sensitive to a 1e-6 statistic, so the absolute tolerance is loose there
    assert res.p_mw[0].item() == pytest.approx(mw.pvalue, rel=2e-3, abs=5e-3)
    assert res.p_kruskal[0].item() == pytest.approx(kw.pvalue, rel=2e-3, abs=5e-3)
    assert res.n_base[0].item() == nb and res.n_cur[0].item() == nc


@SETTINGS
@given(st.integers(2, 30), vals)
def test_constant_samples_never_differ(n, v):
    """All-tied samples: no evidence of a difference (p = 1, no NaN)."""
    B = torch.full((1, n), float(v), dtype=torch.float64)
    C = torch.full((1, n), float(v), dtype=torch.float64)
    res = pairwise.rank_tests(B, C)
    for p in (res.p_mw, res.p_kruskal, res.p_wilcoxon):
        assert not math.isnan(p[0].item()) and p[0].item() > 0.99
    assert not pairwise.pairwise_differs(res, pairwise.PW_ANY, 0.05, 1, 1, 1)[0]


@SETTINGS
@given(st.integers(1, 19), st.integers(1, 19))
def test_short_windows_below_minimum_never_differ(nb, nc):
    """Below MIN_*_DATA_POINTS the tests abstain even for wildly different samples."""
    B = torch.zeros((1, nb), dtype=torch.float64)
    C = torch.full((1, nc), 100.0, dtype=torch.float64)
    res = pairwise.rank_tests(B, C)
    assert not pairwise.pairwise_differs(res, pairwise.PW_ANY, 0.05, 20, 20, 20)[0]


@SETTINGS
@given(st.lists(st.one_of(vals, st.just(float("nan"))), min_size=1, max_size=60))
def test_window_stats_nan_aware(xs):
    y = torch.tensor([xs], dtype=torch.float64)
    s = moving_average.window_stats(y)
    v = np.array(xs)
    v = v[~np.isnan(v)]
    assert int(s.count[0]) == len(v)
    if len(v):
        # the scorer computes in fp32 (as the kernels do)
        assert s.mean[0].item() == pytest.approx(float(np.mean(v)), rel=1e-5, abs=1e-4)
        assert s.std[0].item() == pytest.approx(float(np.std(v)), rel=1e-4, abs=1e-3)


@SETTINGS
@given(st.integers(1, 3), vals, st.floats(0.0, 5.0), st.floats(0.5, 4.0))
def test_detect_bound_semantics(bound, f, sigma, thr):
    """bound bit 1 checks the upper side, bit 2 the lower side; points inside the band never flag."""
    x = torch.tensor([[f + 2 * thr * sigma + 1.0, f - 2 * thr * sigma - 1.0, f]])
    d = detect.detect(torch.full((1, 3), f), torch.tensor([sigma]), x, torch.tensor([thr]),
                      torch.tensor([bound], dtype=torch.int8), torch.tensor([-1e9]))
    hi, lo, mid = d.anomaly[0].tolist()
    assert bool(hi) == bool(bound & 1) and bool(lo) == bool(bound & 2) and not mid
    assert int(d.verdict[0]) == 1


@SETTINGS
@given(st.integers(2, 12), st.integers(2, 6), vals)
def test_decompose_constant_series(m, periods, v):
    y = torch.full((2, m * periods), float(v), dtype=torch.float64)
    d = decompose.seasonal_decompose(y, m)
    ok = ~torch.isnan(d.trend)
    assert torch.allclose(d.trend[ok], torch.full_like(d.trend[ok], float(v)), atol=1e-9)
    assert torch.allclose(d.seasonal, torch.zeros_like(d.seasonal), atol=1e-9)


@SETTINGS
@given(st.text(alphabet=st.characters(blacklist_categories=("Cs",)), max_size=40))
def test_go_query_escape_roundtrip(s):
    from urllib.parse import unquote_plus
    e = urls.go_query_escape(s)
    assert unquote_plus(e) == s
    assert all(ch.isalnum() or ch in "-_.~%+" for ch in e)


@SETTINGS
@given(st.dictionaries(st.from_regex(r"[a-z_][a-z0-9_]{0,8}", fullmatch=True),
                       st.from_regex(r"[a-zA-Z0-9_./-]{0,12}", fullmatch=True), max_size=4))
def test_selector_parse_and_match(labels):
    body = ",".join(f'{k}="{v}"' for k, v in sorted(labels.items()))
    sel = parse_selector("namespace_pod:m{" + body + "}")
    assert sel.name == "namespace_pod:m"
    assert sel.matches(dict(labels, __name__="namespace_pod:m"))
    if labels:
        k = sorted(labels)[0]
        assert not sel.matches(dict(labels, __name__="namespace_pod:m", **{k: labels[k] + "x"}))


@SETTINGS
@given(st.text(max_size=10), st.booleans(), st.integers(0, 10 ** 6),
       st.lists(st.tuples(st.integers(0, 2 ** 40), st.floats(-1e6, 1e6, allow_nan=False)), max_size=4))
def test_monitor_status_go_json_roundtrip(phase, remediated, rev, points):
    s = crd.DeploymentMonitorStatus(phase=phase, remediation_taken=remediated, timestamp="t", expired=False)
    s.anomaly = crd.Anomaly(anomalous_metrics=[crd.AnomalousMetric(
        name="error5xx", values=[crd.AnomalousMetricValue(time=t, value=v) for t, v in points])]) if points \
        else crd.Anomaly()
    enc = to_go(s)
    assert {"phase", "remediationTaken", "timestamp", "expired"} <= set(enc)  # never omitted (no omitempty)
    assert from_go(crd.DeploymentMonitorStatus, enc) == s
