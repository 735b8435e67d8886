"""Wire-format contract tests (golden JSON from the reference Go structs).

Sources: foremast-barrelman/pkg/apis/deployment/v1alpha1/types.go,
foremast-barrelman/pkg/client/analyst/analystclient.go,
foremast-service/pkg/models/models.go, converter.go, prometheushelper.go,
wavefronthelper.go, stringutils.go, elasticsearchstore.go.
"""

import hashlib
import hmac
import json

import httpx
import pytest

from foremast_amd.api import crd, rest, status
from foremast_amd.service import app as svc
from foremast_amd.service import urls
from foremast_amd.store import MemoryJobStore, SqliteJobStore, job_id_for


def test_monitor_json_shape_matches_go():
    m = crd.DeploymentMonitor(metadata={"name": "demo", "namespace": "ns"})
    d = m.to_dict()
    assert d["apiVersion"] == "deployment.foremast.ai/v1alpha1" and d["kind"] == "DeploymentMonitor"
    # structs are never omitted by Go even with omitempty; phase/remediationTaken/timestamp/expired always present
    assert d["spec"] == {"analyst": {"endpoint": ""}, "metrics": {"dataSourceType": "", "endpoint": ""},
                         "remediation": {"option": ""}}
    assert d["status"] == {"phase": "", "remediationTaken": False, "anomaly": {}, "timestamp": "", "expired": False}


def test_monitor_roundtrip_and_unknown_fields():
    raw = {
        "apiVersion": "deployment.foremast.ai/v1alpha1", "kind": "DeploymentMonitor",
        "metadata": {"name": "demo", "namespace": "foremast-examples", "annotations": {"x": "y"}},
        "spec": {"remediation": {"option": "AutoRollback"}, "continuous": True, "rollbackRevision": 3,
                 "metrics": {"dataSourceType": "prometheus", "endpoint": "http://p/api/v1/",
                             "monitoring": [{"metricName": "http_server_requests_error_5xx",
                                             "metricType": "counter", "metricAlias": "error5xx"}]},
                 "futureField": 1},
        "status": {"jobId": "abc", "phase": "Unhealthy", "remediationTaken": True, "timestamp": "t",
                   "expired": False,
                   "anomaly": {"anomalousMetrics": [{"name": "error5xx", "values": [{"time": 1, "value": 2.5}]}]}},
    }
    m = crd.DeploymentMonitor.from_dict(raw)
    assert m.spec.remediation.option == crd.REMEDIATION_AUTO_ROLLBACK
    assert m.spec.metrics.monitoring[0].metric_alias == "error5xx"
    assert m.status.anomaly.anomalous_metrics[0].values[0].value == 2.5
    d = m.to_dict()
    assert "futureField" not in d["spec"]
    assert d["status"]["jobId"] == "abc" and d["spec"]["rollbackRevision"] == 3


def test_constants():
    assert crd.PHASES == ("Healthy", "Running", "Failed", "Unhealthy", "Warning", "Expired", "Abort")
    assert crd.REMEDIATIONS == ("None", "AutoRollback", "AutoPause", "Auto")
    assert crd.CANARY_SUFFIX == "-foremast-canary"


def test_convert_to_anomaly_pairs():
    a = crd.anomaly_from_flat({"error5xx": {"tags": "t", "values": [1700000000, 40.1, 1700000060, 41.0, 99]}})
    vals = a.anomalous_metrics[0].values
    assert [(v.time, v.value) for v in vals] == [(1700000000, 40.1), (1700000060, 41.0)]


@pytest.mark.parametrize("internal,external", [
    ("initial", "new"), ("preprocess_inprogress", "inprogress"), ("postprocess_inprogress", "inprogress"),
    ("preprocess_completed", "inprogress"), ("completed_health", "success"), ("completed_unhealth", "anomaly"),
    ("completed_unknown", "abort"), ("preprocess_failed", "abort"), ("abort", "abort"), ("reprogress", "inprogress"),
    ("whatever", "inprogress"),
])
def test_service_status_map(internal, external):
    assert status.internal_to_external(internal) == external


@pytest.mark.parametrize("ext,phase", [
    ("created", "Running"), ("initial", "Running"), ("new", "Running"), ("inprogress", "Running"),
    ("unknown", "Running"), ("completed_health", "Healthy"), ("success", "Healthy"),
    ("completed_unhealth", "Unhealthy"), ("anomaly", "Unhealthy"), ("abort", "Abort"),
    ("completed_unknown", "Warning"), ("zzz", "zzz"),
])
def test_barrelman_phase_map(ext, phase):
    assert status.external_to_phase(ext) == phase


def _mq(endpoint="http://prometheus:9090/api/v1/", query='namespace_pod:m{namespace="ns",pod="p-1"}',
        start=1700000040, end=1700000700, step=60):
    return rest.MetricQuery(data_source_type="prometheus",
                            parameters={"endpoint": endpoint, "query": query, "start": start, "end": end, "step": step})


def test_prometheus_url_is_go_compatible():
    u = urls.build_prometheus_url(_mq(query='a:b{x="1 2",y=~"p|q"}'))
    assert u == ("http://prometheus:9090/api/v1/query_range?query=a%3Ab%7Bx%3D%221+2%22%2Cy%3D~%22p%7Cq%22%7D"
                 "&start=1700000040&end=1700000700&step=60")
    p = urls.parse_prometheus_url(u)
    assert p["query"] == 'a:b{x="1 2",y=~"p|q"}' and p["step"] == 60


def test_wavefront_url():
    q = rest.MetricQuery(data_source_type="wavefront", parameters={"query": "ts(x)", "start": 10, "end": 70, "step": 60})
    assert urls.build_wavefront_url(q) == "ts%28x%29&&10&&m&&70"
    assert urls.parse_wavefront_url("ts%28x%29&&10&&m&&70")["query"] == "ts(x)"


def test_config_string_roundtrip_sorted():
    code, cfg, stores = urls.flatten_queries({"b": _mq(), "a": _mq(step=30)})
    assert code == 0
    assert cfg.startswith("a== http") and " ||b== http" in cfg
    assert stores == "a== prometheus ||b== prometheus"
    parsed = urls.parse_config(cfg)
    assert set(parsed) == {"a", "b"} and parsed["a"].endswith("step=30")


def test_job_id_is_hmac_sha256_empty_key():
    d = rest.DocumentRequest(app_name="demo", start_time="2020-01-01T00:00:00Z", end_time="2020-01-01T00:10:00Z",
                             current_config="c", strategy="canary")
    exp = hmac.new(b"", b"demo2020-01-01T00:00:00Z2020-01-01T00:10:00Zccanary", hashlib.sha256).hexdigest()
    assert job_id_for(d) == exp


def _req(strategy="canary", **kw):
    return {"appName": "demo", "startTime": "2020-01-01T00:00:00Z", "endTime": "2020-01-01T00:10:00Z",
            "strategy": strategy,
            "metrics": {"current": {"error5xx": {"dataSourceType": "prometheus", "parameters": {
                "endpoint": "http://prometheus:9090/api/v1/", "query": 'namespace_pod:x{namespace="ns",pod="p"}',
                "start": 1577836860, "end": 1577837460, "step": 60}}}, **kw}}


def _make_store(kind, tmp_path):
    if kind == "memory":
        return MemoryJobStore()
    if kind == "sqlite":
        return SqliteJobStore(str(tmp_path / "jobs.db"))
    import httpx
    from foremast_amd.store.es import ElasticJobStore
    from foremast_amd.store.fake_es import FakeElasticsearch
    return ElasticJobStore("http://es:9200", transport=httpx.WSGITransport(app=FakeElasticsearch()))


@pytest.mark.parametrize("store_kind", ["memory", "sqlite", "es"])
def test_register_and_lookup(tmp_path, store_kind):
    store = _make_store(store_kind, tmp_path)
    code, body = svc.register(store, _req())
    assert code == 200 and body["status"] == "new" and body["statusCode"] == 200 and "reason" not in body
    code2, body2 = svc.register(store, _req())
    assert body2["jobId"] == body["jobId"]  # idempotent
    assert len(store.all()) == 1
    doc = store.get(body["jobId"])
    assert doc["status"] == "initial" and doc["currentConfig"].startswith("error5xx== http")
    assert set(rest.DOCUMENT_FIELDS) <= set(doc)
    look = svc.lookup(store, body["jobId"])
    assert look == {"jobId": body["jobId"], "statusCode": 200, "status": "new", "anomaly": None}
    store.update(body["jobId"], {"status": "completed_unhealth", "reason": "spike",
                                 "anomalyInfo": json.dumps({"error5xx": {"tags": "", "values": [1577836920, 40.5]}})})
    look = svc.lookup(store, body["jobId"])
    assert look["status"] == "anomaly" and look["reason"] == "spike"
    assert look["anomaly"]["error5xx"]["values"] == [1577836920, 40.5]
    missing = svc.lookup(store, "nope")
    assert missing == {"jobId": "nope", "statusCode": 200, "status": "unknown", "reason": "nope not found."}


def test_register_validation():
    store = MemoryJobStore()
    assert svc.register(store, [1])[0] == 400
    bad = _req()
    bad["appName"] = "  "
    assert svc.register(store, bad) == (400, {"error": "appName is empty"})
    nocur = _req()
    nocur["metrics"]["current"] = {}
    code, body = svc.register(store, nocur)
    assert code == 400 and "current is empty" in body["error"]
    badtime = _req()
    badtime["startTime"] = "yesterday"
    code, body = svc.register(store, badtime)
    assert code == 400  # the reference log.Fatal()s here (Q5)
    wrongsrc = _req()
    wrongsrc["metrics"]["current"]["error5xx"]["dataSourceType"] = "graphite"
    assert svc.register(store, wrongsrc)[0] == 400


def test_service_http_and_proxy():
    import asyncio
    from foremast_amd.promql.fake import FakePrometheus
    from foremast_amd.promql import synth

    prom = FakePrometheus(clock=lambda: 1_700_000_600)
    prom.add("namespace_app_per_pod:m", {"namespace": "ns", "app": "demo"}, synth.seasonal(noise=0))
    app = svc.create_app(MemoryJobStore(), query_endpoint="http://prom:9090/",
                         proxy_transport=httpx.ASGITransport(app=prom.asgi_app()))

    async def go():
        async with httpx.AsyncClient(transport=httpx.ASGITransport(app=app), base_url="http://svc") as c:
            r = await c.post("/v1/healthcheck/create", content=json.dumps(_req()))
            assert r.status_code == 200
            jid = r.json()["jobId"]
            r = await c.get(f"/v1/healthcheck/id/{jid}")
            assert r.json()["status"] == "new"
            r = await c.post("/v1/healthcheck/create", content=b"{not json")
            assert r.status_code == 400 and r.json() == {"error": "Bad request"}
            q = "query=namespace_app_per_pod%3Am%7Bapp%3D%22demo%22%7D&start=1700000000&end=1700000600&step=60"
            r = await c.get("/api/v1/query_range?" + q)
            assert r.headers["access-control-allow-origin"] == "*"
            inner = json.loads(r.json())  # double-encoded, as the UI expects (Q1)
            assert inner["status"] == "success" and len(inner["data"]["result"][0]["values"]) == 11
            r = await c.get("/api/v1/query_range?" + q + "&raw=1")
            assert r.json()["status"] == "success"
    asyncio.run(go())


@pytest.mark.parametrize("store_kind", ["memory", "sqlite", "es"])
def test_store_claim_lease_semantics(tmp_path, store_kind):
    """Claims are exclusive, stuck jobs are taken over after MAX_STUCK_IN_SECONDS,
    and a worker that lost its lease cannot overwrite the new owner's result."""
    store = _make_store(store_kind, tmp_path)
    ids = [svc.register(store, _req(strategy=s))[1]["jobId"] for s in ("canary", "rollover", "continuous")]
    a = store.claim("A", now=1000.0, limit=2)
    b = store.claim("B", now=1000.0)
    got_a, got_b = {d["id"] for d in a}, {d["id"] for d in b}
    assert len(got_a) == 2 and len(got_b) == 1 and not (got_a & got_b) and (got_a | got_b) == set(ids)
    assert store.claim("C", now=1010.0) == []            # in progress, not stuck yet
    stolen = store.claim("C", now=10_000.0, max_stuck_s=90.0)
    assert {d["id"] for d in stolen} == set(ids)          # stuck-job takeover
    jid = a[0]["id"]
    assert not store.update(jid, {"status": "completed_health"}, expect_claimed_by="A")
    assert store.update(jid, {"status": "completed_health"}, expect_claimed_by="C")
    assert store.get(jid)["status"] == "completed_health"


def test_es_store_conflicts_and_faults():
    import httpx
    from foremast_amd.store.es import ElasticJobStore
    from foremast_amd.store.fake_es import FakeElasticsearch
    from foremast_amd.store.jobstore import open_store
    fake = FakeElasticsearch()
    s1 = ElasticJobStore("http://es:9200", transport=httpx.WSGITransport(app=fake))
    s2 = ElasticJobStore("http://es:9200", transport=httpx.WSGITransport(app=fake))
    assert s1.all() == [] and s1.claim("x") == []        # index does not exist yet
    jid = svc.register(s1, _req())[1]["jobId"]
    assert s2.get(jid)["status"] == "initial"
    # interleaved read-modify-write: s2's stale version is rejected, then retried
    d, v = s1._get_versioned(jid)
    assert s2.update(jid, {"reason": "from s2"})
    d["reason"] = "stale"
    assert not s1._put_versioned(d, v)
    assert s1.get(jid)["reason"] == "from s2"
    fake.fail_next = 1
    with pytest.raises(httpx.HTTPStatusError):
        s1.get(jid)
    s1.wait_ready(deadline_s=1.0)
    assert isinstance(open_store("http://es:9200"), ElasticJobStore)


def test_dashboard_page():
    from fastapi.testclient import TestClient
    from foremast_amd.service import ui
    store = MemoryJobStore()
    svc.register(store, _req())
    client = TestClient(svc.create_app(store, query_endpoint="http://prom:9090/"))
    r = client.get("/ui/foremast-examples/demo")
    assert r.status_code == 200 and r.headers["content-type"].startswith("text/html")
    body = r.text
    q = ui.queries("foremast-examples", "demo")
    upper = q["http_server_requests_error_5xx"]["upper"]
    assert "foremastbrain:namespace_app_per_pod:http_server_requests_error_5xx_upper" in upper
    assert "exported_namespace" in body and "/api/v1/query_range?query=" in body and "<script>" in body
    idx = client.get("/ui")
    assert "demo" in idx.text
    xss = client.get("/ui/%3Cscript%3E/x")
    assert "<script>alert" not in xss.text and "&lt;script&gt;" in xss.text
