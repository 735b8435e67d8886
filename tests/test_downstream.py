"""Downstream impact (reference README.md:24; the metrics starter's ``caller``
tag, CallerWebMvcTagsProvider.java:22-25): a rollout that degrades the latency
seen by ONE calling service is detected on that caller's series, scored jointly
(latency + error rate) per caller, and the DeploymentMonitor names the caller."""

import asyncio
import json

import httpx
import pytest

from foremast_amd.api import crd
from foremast_amd.brain.batch import BatchScorer
from foremast_amd.brain.worker import BrainWorker
from foremast_amd.controller import queries
from foremast_amd.controller.analyst import AnalystClient
from foremast_amd.controller.barrelman import Barrelman
from foremast_amd.deploy import rules
from foremast_amd.k8s.fake import FakeCluster
from foremast_amd.promql import synth
from foremast_amd.promql.client import PromClient
from foremast_amd.promql.fake import FakePrometheus
from foremast_amd.service.app import create_app
from foremast_amd.store import MemoryJobStore
from foremast_amd.utils.config import BrainConfig, reference_default_env

NS = "shop"
T0 = 1_700_000_000.0
LAT = "http_server_requests_latency"
ERR = "http_server_requests_errors"
CALLERS = ("web", "batch")


class Clock:
    def __init__(self, t):
        self.t = t

    def __call__(self):
        return self.t


def _metadata():
    mon = [{"metricName": LAT, "metricType": "downstream", "metricAlias": "latency"},
           {"metricName": ERR, "metricType": "downstream", "metricAlias": "errors"}]
    return {"apiVersion": "deployment.foremast.ai/v1alpha1", "kind": "DeploymentMetadata",
            "metadata": {"name": "spring-boot", "namespace": "foremast"},
            "spec": {"analyst": {"endpoint": "http://foremast-service:8099/v1/healthcheck/"},
                     "metrics": {"dataSourceType": "prometheus", "endpoint": "http://prometheus:9090/api/v1/",
                                 "monitoring": mon}}}


def test_caller_queries_and_rules():
    md = crd.DeploymentMetadata.from_dict(_metadata())
    q = queries.create_map(NS, "cart", ["cart-v2-a", "cart-v2-b"], md.spec.metrics, r_cat("current"), 10,
                           "rollingupdate", now=T0)
    assert q["latency"].parameters["query"].startswith("namespace_pod_caller:" + LAT + "{")
    h = queries.create_map(NS, "cart", [], md.spec.metrics, r_cat("historical"), 10, "rollingupdate", now=T0)
    assert h["errors"].parameters["query"] == f'namespace_app_caller_per_pod:{ERR}{{namespace="{NS}",app="cart"}}'
    names = set(rules.recorded_names())
    for fam in rules.HTTP_FAMILIES:
        for pfx in rules.CALLER_PREFIX.values():
            assert pfx + fam in names
    per_pod = [r for r in rules.rules() if r["record"] == "namespace_app_caller_per_pod:" + LAT][0]
    assert "group_left" in per_pod["expr"]  # many (callers) to one (pod count)


def r_cat(name):
    from foremast_amd.api import rest
    return {"current": rest.CATEGORY_CURRENT, "historical": rest.CATEGORY_HISTORICAL}[name]


def _world(device):
    import torch
    clock = Clock(T0)
    kube = FakeCluster()
    for ns in (NS, "foremast"):
        kube.add_namespace(ns)
    kube.create_sync("deploymentmetadatas", _metadata())
    prom = FakePrometheus(clock=clock)
    for i, c in enumerate(CALLERS):  # 7-day per-caller history of the app
        lab = {"namespace": NS, "app": "cart", "caller": c}
        prom.add("namespace_app_caller_per_pod:" + LAT, lab,
                 synth.seasonal(level=0.10 + 0.05 * i, amp=0.02, noise=0.003, seed=10 + i))
        prom.add("namespace_app_caller_per_pod:" + ERR, lab, synth.error_rate(base=0.3, spread=0.1, seed=20 + i))
    store = MemoryJobStore()
    svc_transport = httpx.ASGITransport(app=create_app(store, query_endpoint="http://prometheus:9090/"))
    barrel = Barrelman(kube, namespace="foremast", clock=clock, poll_seconds=0, pod_retry_sleep=0,
                       analyst_factory=lambda ep: AnalystClient(ep, transport=svc_transport))
    env = reference_default_env()
    env.update(ML_ALGORITHM="holt_winters", MIN_HISTORICAL_DATA_POINT_TO_MEASURE="10")
    cfg = BrainConfig.from_env(env)
    brain = BrainWorker(store, cfg, prom=PromClient(transport=httpx.ASGITransport(app=prom.asgi_app())),
                        scorer=BatchScorer(cfg, device=torch.device(device)), worker_id="brain-0", clock=clock)
    return clock, kube, prom, store, barrel, brain


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_rollout_degrading_one_caller_names_it(device):
    clock, kube, prom, store, barrel, brain = _world(device)

    async def go():
        v1 = kube.apply_deployment(NS, "cart", "cart", "shop/cart:v1", replicas=2, labels={"appType": "spring-boot"})
        await barrel.on_deployment_added(v1)
        old_hash = kube.list_sync("replicasets", NS)[0]["metadata"]["labels"]["pod-template-hash"]
        v1 = kube.get_sync("deployments", NS, "cart")
        v2 = kube.apply_deployment(NS, "cart", "cart", "shop/cart:v2", replicas=2, labels={"appType": "spring-boot"})
        for j, p in enumerate(sorted(kube.list_sync("pods", NS), key=lambda p: p["metadata"]["name"])):
            new = p["metadata"]["labels"]["pod-template-hash"] != old_hash
            for i, c in enumerate(CALLERS):
                lab = {"namespace": NS, "pod": p["metadata"]["name"], "caller": c}
                lat = synth.seasonal(level=0.10 + 0.05 * i, amp=0.02, noise=0.003, seed=100 + 7 * j + i)
                if new and c == "batch":  # v2 regresses only the API the batch caller uses
                    lat = synth.step_change(lat, at=T0 + 120, factor=3.0)
                prom.add("namespace_pod_caller:" + LAT, lab, lat)
                prom.add("namespace_pod_caller:" + ERR, lab, synth.error_rate(base=0.3, spread=0.1, seed=200 + j))
        await barrel.on_deployment_updated(v1, v2)
        await barrel.drain()
        mon = crd.DeploymentMonitor.from_dict(kube.get_sync("deploymentmonitors", NS, "cart"))
        doc = store.get(mon.status.job_id)
        assert "namespace_pod_caller%3A" + LAT in doc["currentConfig"]
        clock.t = T0 + 300
        assert await brain.cycle() == 1
        doc = store.get(mon.status.job_id)
        assert doc["status"] == "completed_unhealth", doc["reason"]
        info = json.loads(doc["anomalyInfo"])
        assert "latency[caller=batch]" in info, info.keys()
        assert not any("caller=web" in k for k in info), info.keys()
        assert info["latency[caller=batch]"]["tags"].startswith("caller=batch")
        assert min(info["latency[caller=batch]"]["values"][1::2]) > 0.2  # the x3 latency
        await barrel.check_running_status()
        m2 = crd.DeploymentMonitor.from_dict(kube.get_sync("deploymentmonitors", NS, "cart"))
        assert m2.status.phase == crd.PHASE_UNHEALTHY
        names = [a.name for a in m2.status.anomaly.anomalous_metrics]
        assert "latency[caller=batch]" in names
        assert any("caller=batch" in a.tags for a in m2.status.anomaly.anomalous_metrics)
        # the joint per-caller model ran (one cached model per caller with >= 2 metrics)
        assert brain.downstream is not None and len(brain.downstream.cache) == len(CALLERS)
        assert brain.downstream.fp8

    asyncio.run(go())


def test_per_caller_continuous_jobs_stay_with_the_batch_worker():
    from foremast_amd.brain.streaming import is_streamable
    from foremast_amd.service import app as svc
    from foremast_amd.utils.timeutil import format_rfc3339
    store = MemoryJobStore()

    def job(metric, app):
        q = f'{metric}{{namespace="{NS}",app="{app}"}}'
        p = {"endpoint": "http://prometheus:9090/api/v1/", "query": q, "step": 60}
        m = {"latency": {"dataSourceType": "prometheus", "parameters": dict(p, start=int(T0), end=int(T0 + 600))}}
        return {"appName": app, "startTime": format_rfc3339(T0), "endTime": format_rfc3339(T0 + 600),
                "strategy": "continuous", "metrics": {"current": m, "historical": m}}
    a = svc.register(store, job("namespace_app_per_pod:" + LAT, "a"))[1]["jobId"]
    b = svc.register(store, job("namespace_app_caller_per_pod:" + LAT, "b"))[1]["jobId"]
    assert is_streamable(store.get(a)) and not is_streamable(store.get(b))
    w = BrainWorker(store, BrainConfig(), exclude_strategies=("continuous",))
    assert [d["id"] for d in store.claim("w", now=T0, max_stuck_s=90, only=w._claimable)] == [b]


def test_api_level_rollup_names_the_request_path():
    """``metricType: api`` (reference README.md:26, anomalies aggregated at service
    or API level): the same families per request path (``uri``); a v2 that fails
    one endpoint is reported on that path only."""
    import torch
    clock = Clock(T0)
    kube = FakeCluster()
    for ns in (NS, "foremast"):
        kube.add_namespace(ns)
    md = _metadata()
    md["spec"]["metrics"]["monitoring"] = [{"metricName": ERR, "metricType": "api", "metricAlias": "errors"}]
    kube.create_sync("deploymentmetadatas", md)
    prom = FakePrometheus(clock=clock)
    paths = ("/orders", "/cart")
    for i, u in enumerate(paths):
        prom.add("namespace_app_uri_per_pod:" + ERR, {"namespace": NS, "app": "cart", "uri": u},
                 synth.error_rate(base=0.3, spread=0.1, seed=40 + i))
    store = MemoryJobStore()
    svc_transport = httpx.ASGITransport(app=create_app(store, query_endpoint="http://prometheus:9090/"))
    barrel = Barrelman(kube, namespace="foremast", clock=clock, poll_seconds=0, pod_retry_sleep=0,
                       analyst_factory=lambda ep: AnalystClient(ep, transport=svc_transport))
    env = reference_default_env()
    env.update(ML_ALGORITHM="moving_average_all", MIN_HISTORICAL_DATA_POINT_TO_MEASURE="10")
    cfg = BrainConfig.from_env(env)
    brain = BrainWorker(store, cfg, prom=PromClient(transport=httpx.ASGITransport(app=prom.asgi_app())),
                        scorer=BatchScorer(cfg, device=torch.device("cpu")), worker_id="brain-0", clock=clock)

    async def go():
        v1 = kube.apply_deployment(NS, "cart", "cart", "shop/cart:v1", replicas=1, labels={"appType": "spring-boot"})
        await barrel.on_deployment_added(v1)
        old_hash = kube.list_sync("replicasets", NS)[0]["metadata"]["labels"]["pod-template-hash"]
        v1 = kube.get_sync("deployments", NS, "cart")
        v2 = kube.apply_deployment(NS, "cart", "cart", "shop/cart:v2", replicas=1, labels={"appType": "spring-boot"})
        for j, p in enumerate(kube.list_sync("pods", NS)):
            new = p["metadata"]["labels"]["pod-template-hash"] != old_hash
            for i, u in enumerate(paths):
                gen = synth.error_rate(base=0.3, spread=0.1, seed=60 + 3 * j + i)
                if new and u == "/orders":
                    gen = synth.step_change(gen, at=T0 + 120, factor=0.0, add=25.0)
                prom.add("namespace_pod_uri:" + ERR, {"namespace": NS, "pod": p["metadata"]["name"], "uri": u}, gen)
        await barrel.on_deployment_updated(v1, v2)
        await barrel.drain()
        mon = crd.DeploymentMonitor.from_dict(kube.get_sync("deploymentmonitors", NS, "cart"))
        assert "namespace_pod_uri%3A" + ERR in store.get(mon.status.job_id)["currentConfig"]
        clock.t = T0 + 300
        assert await brain.cycle() == 1
        doc = store.get(mon.status.job_id)
        assert doc["status"] == "completed_unhealth"
        info = json.loads(doc["anomalyInfo"])
        assert list(info) == ["errors[uri=/orders]"] and info["errors[uri=/orders]"]["tags"].startswith("uri=/orders")

    asyncio.run(go())
