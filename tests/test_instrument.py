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
