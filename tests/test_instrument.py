"""App-side instrumentation (starter equivalent) and the demo fault injector."""

import asyncio
import os
import sys

import httpx

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "examples", "demo"))

from foremast_amd.instrument import ForemastMetrics, parse_common_tags  # noqa: E402


def test_common_tags_env_and_fallback():
    assert parse_common_tags("app:ENV.APP_NAME|info.app.name", {"APP_NAME": "demo"}) == {"app": "demo"}
    assert parse_common_tags("app:ENV.APP_NAME|fallback", {}) == {"app": "fallback"}


def test_middleware_exposition_matches_recording_rules():
    import app as demo
    mw = demo.build_app("demo")

    async def go():
        async with httpx.AsyncClient(transport=httpx.ASGITransport(app=mw), base_url="http://d") as c:
            assert (await c.get("/")).status_code == 200
            assert (await c.get("/error5xx", headers={"X-CALLER": "checkout"})).status_code == 500
            assert (await c.get("/nope")).status_code == 404
            return (await c.get("/actuator/prometheus")).text

    text = asyncio.run(go())
    lines = [ln for ln in text.splitlines() if ln.startswith("http_server_requests_seconds_count{")]
    assert any('status="500"' in ln and 'app="demo"' in ln and 'caller="checkout"' in ln and ln.endswith(" 1.0")
               for ln in lines)
    assert any('status="200"' in ln and 'uri="/"' in ln for ln in lines)
    # pre-registered zero series for the starter's default statuses
    for st in ("403", "501", "502"):
        assert any(f'status="{st}"' in ln and ln.endswith(" 0.0") for ln in lines), st
    assert "http_server_requests_seconds_sum{" in text and "http_server_requests_seconds_max{" in text
    assert "_total" not in "".join(lines)


def test_fault_injector_replays_rates():
    import app as demo
    mw = demo.build_app("demo")
    rates = demo.read_rates(os.path.join(ROOT, "examples", "demo", "data", "spike_rates.txt"))
    assert len(rates) == 60 and max(rates) > 40 and sorted(rates)[len(rates) // 2] < 1

    async def go():
        async with httpx.AsyncClient(transport=httpx.ASGITransport(app=mw), base_url="http://d") as c:
            inj = demo.FaultInjector(c, "5xx", rates=[2.0, 0.0, 5.0], tick=1.0, speed=50.0)
            await inj.run(asyncio.Event())
            return inj.sent

    assert asyncio.run(go()) == 7
    assert isinstance(mw, ForemastMetrics) and mw.count_of(500) == 7


def test_common_metrics_filter_semantics():
    """CommonMetricsFilter.java: overrides (longest dotted prefix, then 'all'),
    whitelist, blacklist, prefixes; runtime enable/disable moves a meter
    between the lists; names compare in Micrometer's dotted form."""
    from foremast_amd.instrument import CommonMetricsFilter, meter_name
    assert meter_name("http_server_requests_seconds") == "http.server.requests"
    assert meter_name("http_server_requests_seconds_max") == "http.server.requests"
    assert meter_name("jvm_memory_used_bytes") == "jvm.memory.used"
    off = CommonMetricsFilter(enabled=False, blacklist="http_server_requests")
    assert off.accept("http_server_requests_seconds")  # disabled filter shows everything
    f = CommonMetricsFilter(enabled=True, whitelist="jvm_memory_used", blacklist="http_server_requests",
                            prefixes="process,http")
    assert f.accept("jvm_memory_used_bytes")
    assert not f.accept("http_server_requests_seconds")  # blacklist beats the 'http' prefix
    assert f.accept("http_client_requests_seconds") and f.accept("process_cpu_usage")
    assert not f.accept("system_load_average_1m")
    f.enable_metric("http_server_requests")
    assert f.accept("http_server_requests_seconds")
    f.disable_metric("jvm.memory.used")
    assert not f.accept("jvm_memory_used_bytes")
    o = CommonMetricsFilter(enabled=True, enable_overrides={"jvm": False, "all": True})
    assert not o.accept("jvm_memory_used_bytes") and o.accept("anything_else")


def test_metrics_actuator_toggles_exposition():
    """/actuator/k8s-metrics/{disable,enable}/<metric> hides / shows a meter in
    the Prometheus exposition (K8sMetricsEndpoint.java)."""
    from prometheus_client import CollectorRegistry, Counter
    from foremast_amd.instrument import CommonMetricsFilter

    async def inner(scope, receive, send):
        await send({"type": "http.response.start", "status": 200, "headers": []})
        await send({"type": "http.response.body", "body": b"ok"})

    reg = CollectorRegistry()
    Counter("orders_placed", "orders", registry=reg).inc(3)
    mw = ForemastMetrics(inner, app_name="demo", registry=reg,
                         metrics_filter=CommonMetricsFilter(enabled=True, prefixes="http,orders"))

    async def go():
        async with httpx.AsyncClient(transport=httpx.ASGITransport(app=mw), base_url="http://d") as c:
            await c.get("/")
            t0 = (await c.get("/actuator/prometheus")).text
            r = await c.get("/actuator/k8s-metrics/disable/orders_placed")
            t1 = (await c.get("/actuator/prometheus")).text
            await c.get("/actuator/k8s-metrics/enable/orders_placed")
            t2 = (await c.get("/actuator/prometheus")).text
            return t0, r, t1, t2

    t0, r, t1, t2 = asyncio.run(go())
    assert r.status_code == 200 and r.text == "OK"
    assert "orders_placed_total 3.0" in t0 and "http_server_requests_seconds_count" in t0
    assert "orders_placed" not in t1 and "http_server_requests_seconds_count" in t1
    assert "orders_placed_total 3.0" in t2


def test_dashboard_has_error_latency_scatter():
    from foremast_amd.service import ui
    pg = ui.page("ns", "demo")
    assert "drawScatter" in pg and '"scatter": ["http_server_requests_error_5xx", "http_server_requests_latency"]' in pg
