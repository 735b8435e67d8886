"""The native rollout-job decoder (ingest/csrc/job_plan.cpp) against the Python
parser (brain/plans.py ``_plan``): identical plans on every document the native
decoder accepts, declines (never a different plan) on everything else."""

import random

import numpy as np
import pytest

from foremast_amd.api import crd
from foremast_amd.api import rest as r
from foremast_amd.brain import plans as P
from foremast_amd.controller import queries
from foremast_amd.ingest import native
from foremast_amd.service import app as svc
from foremast_amd.store import MemoryJobStore
from foremast_amd.utils.timeutil import format_rfc3339

T0 = 1_700_000_040.0
EP = "http://prometheus:9090/api/v1/"
METRICS = (("http_server_requests_error_5xx", "error5xx"), ("http_server_requests_latency", "latency"),
           ("http_server_requests_count", "count"))


def docs_for(n, strategy="canary", rng=None):
    rng = rng or random.Random(0)
    store = MemoryJobStore()
    out = []
    for i in range(n):
        mets = crd.Metrics(data_source_type="prometheus", endpoint=EP,
                           monitoring=[crd.Monitoring(metric_name=m, metric_alias=a) for m, a in METRICS])
        app, ns = f"app-{i}", f"ns{i % 7}"
        new = [f"{app}-v2-{k}-{rng.randrange(1 << 20):05x}" for k in range(rng.randint(1, 6))]
        old = [f"{app}-v1-{k}-{rng.randrange(1 << 20):05x}" for k in range(rng.randint(1, 6))]
        info = queries.create_metrics_info(ns, app, [new, old], mets, rng.choice([5, 10, 30]),
                                           strategy, now=T0 + 60 * i)
        req = r.ApplicationHealthAnalyzeRequest(app_name=app, start_time=format_rfc3339(T0 + 60 * i),
                                                end_time=format_rfc3339(T0 + 60 * i + 600), metrics=info,
                                                strategy=strategy).to_dict()
        code, resp = svc.register(store, req)
        assert code == 200
        out.append(store.get(resp["jobId"]))
    return out


def same(a, b):
    assert a.doc_id == b.doc_id and a.app == b.app and a.end_ts == b.end_ts
    assert len(a.series) == len(b.series)
    for x, y in zip(a.series, b.series):
        assert x == y, (x, y)


def check(docs, expect_native=None):
    nat = P._native_batch(docs, 60.0, 11)
    assert nat is not None
    ok, plans = nat
    for d, acc, p in zip(docs, ok, plans):
        ref = P._plan(d, 60.0, 11)
        if acc:
            assert ref is not None, d
            same(p, ref)
            # the keys the engine indexes by, against the Python hash of the same strings
            c, s0 = p.cols, p.s0
            for k, s in enumerate(ref.series):
                assert int(c.u64[s0 + k, 0]) == P.hkey_hash(s.hkey)
                assert int(c.u64[s0 + k, 1]) == native.key_hash(*s.fam)
                assert int(c.u64[s0 + k, 3]) == native.key_hash(s.hkey[0], s.hkey[1])
                assert int(c.u64[s0 + k, 4]) == native.key_hash(s.hkey[2], s.hkey[3])
                q0, nq = int(c.i32[s0 + k, 2]), int(c.i32[s0 + k, 3])
                assert c.pod_u64[q0:q0 + nq].tolist() == native.key_hashes(
                    [s.namespace] * nq, list(s.cur_pods)).tolist()
    if expect_native is not None:
        assert bool(ok.all()) == expect_native
    return ok


@pytest.mark.parametrize("strategy", ["canary", "rollingUpdate"])
def test_native_plan_equals_python_on_barrelman_jobs(strategy):
    ok = check(docs_for(40, strategy), expect_native=True)
    assert ok.all()


def test_native_plan_declines_or_agrees_on_mutations():
    rng = random.Random(7)
    base = docs_for(30, rng=rng)
    muts = []
    fields = ["currentConfig", "baselineConfig", "historicalConfig", "endTime", "strategy"]
    edits = [
        lambda s: s.replace("%7C", "|"), lambda s: s.replace("%22", '"'), lambda s: s.replace("%3D", "%3d"),
        lambda s: s.replace("start=", "start=+"), lambda s: s.replace("&step=60", "&step=60.0"),
        lambda s: s.replace("&step=60", "&step=30"), lambda s: s.replace("&step=60", "&step=6e1"),
        lambda s: s.replace(" ||", " ||  "), lambda s: s.replace("== ", "==  "), lambda s: s.replace("pod%3D~", "pod%3D"),
        lambda s: s.replace("app%3D%22", "app%3D~%22"), lambda s: s.replace("Z", "+00:00"),
        lambda s: s.replace("canary", "CaNaRy"), lambda s: s.replace("%2C", "%2C%20"),
        lambda s: s.replace("namespace_pod%3A", "namespace_pod_caller%3A"), lambda s: s + " ||x== y",
        lambda s: s.replace("%7D", "%7D%0A"), lambda s: s.replace("-v2-", "-v2%2E"), lambda s: s.replace("0&", "0&&"),
        lambda s: s.replace("query=", "query=%E2%9C%93"), lambda s: s.replace("T", "t"), lambda s: s[:-3],
        lambda s: s.replace("%7C", "%7C%7C"), lambda s: s.replace("http", "HTTP"), lambda s: "",
    ]
    for d in base:
        for _ in range(6):
            m = dict(d)
            f = rng.choice(fields)
            if isinstance(m.get(f), str):
                m[f] = rng.choice(edits)(m[f])
            m["id"] = f"{d['id']}-{len(muts)}"
            muts.append(m)
    ok = check(muts)
    assert 0 < ok.sum() < len(muts)  # both paths exercised


def test_plan_many_memoises_and_mixes_paths():
    docs = docs_for(5)
    odd = dict(docs[1], id="odd", currentConfig=docs[1]["currentConfig"].replace("&step=60", "&step=60.0"))
    got = P.plan_many(docs + [odd, dict(docs[0], id="cont", strategy="continuous")], "holt_winters")
    assert got[-1] is None and got[5] is not None and got[5].series[0].cur_n == 11
    again = P.plan_many(docs, "holt_winters")
    assert all(a is b for a, b in zip(again, got[:5]))
    # lstm / auto / bivariate_normal jobs are keyed too (joint models on the resident engine)
    assert all(p is not None for p in P.plan_many(docs, "lstm"))
    assert P.plan_many(docs, "no_such_algorithm") == [None] * 5


def test_native_plan_throughput():
    import time
    docs = docs_for(400)
    t0 = time.perf_counter()
    nat = P._native_batch(docs, 60.0, 11)
    dt = (time.perf_counter() - t0) / len(docs)
    assert nat[0].all()
    assert dt < 60e-6, f"{dt * 1e6:.1f} us per job"
