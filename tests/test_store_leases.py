"""Job-store claim indexes and worker-heartbeat leases (all three backends)."""

import httpx
import pytest

from foremast_amd.api import rest as r
from foremast_amd.store import MemoryJobStore, SqliteJobStore
from foremast_amd.store.es import ElasticJobStore
from foremast_amd.store.fake_es import FakeElasticsearch


def _store(kind, tmp_path):
    if kind == "memory":
        return MemoryJobStore()
    if kind == "sqlite":
        return SqliteJobStore(str(tmp_path / "jobs.db"))
    es = FakeElasticsearch()
    if kind == "es-keyword":  # an operator-created index: the lease fields mapped `keyword` explicitly
        status, _ = es.handle("PUT", "/documents", {}, {"mappings": {"document": {"properties": {
            "status": {"type": "keyword"}, "claimed_by": {"type": "keyword"}, "id": {"type": "keyword"}}}}})
        assert status == 200
    return ElasticJobStore("http://es:9200", transport=httpx.WSGITransport(app=es))


KINDS = ["memory", "sqlite", "es", "es-keyword"]


def _req(i):
    return r.DocumentRequest(app_name=f"app{i}", start_time="2023-11-14T22:13:20Z", end_time="2023-11-14T22:23:20Z",
                             current_config=f"m== http://p/api/v1/query_range?query=x{i}", strategy="canary")


@pytest.mark.parametrize("kind", KINDS)
def test_heartbeat_keeps_leases_alive(kind, tmp_path):
    st = _store(kind, tmp_path)
    ids = [st.create(_req(i), now=1000.0) for i in range(6)]
    got = st.claim("A", now=1000.0, limit=4)
    assert len(got) == 4
    # A renews ALL its leases with one heartbeat; its jobs are not stuck at +120 s
    st.heartbeat("A", now=1100.0)
    b = st.claim("B", now=1120.0, max_stuck_s=90.0)
    assert sorted(d["id"] for d in b) == sorted(set(ids) - {d["id"] for d in got})  # only the 2 open ones
    # A stops beating: after max_stuck its jobs move to C (B's were claimed at 1120, still fresh)
    c = st.claim("C", now=1195.0, max_stuck_s=90.0)
    assert sorted(d["id"] for d in c) == sorted(d["id"] for d in got)
    # steal_from moves a live holder's jobs at once
    d = st.claim("D", now=1196.0, steal_from={"B"})
    assert sorted(x["id"] for x in d) == sorted(x["id"] for x in b)


@pytest.mark.parametrize("kind", KINDS)
def test_update_many_respects_leases(kind, tmp_path):
    st = _store(kind, tmp_path)
    ids = [st.create(_req(i), now=1000.0) for i in range(3)]
    st.claim("A", now=1000.0, limit=2)
    held = [d["id"] for d in st.all() if d.get("claimed_by") == "A"]
    free = [i for i in ids if i not in held][0]
    res = st.update_many([(held[0], {"status": r.ST_COMPLETED_HEALTH}), (free, {"status": r.ST_COMPLETED_HEALTH})],
                         expect_claimed_by="A")
    assert res == [True, False]
    assert st.get(held[0])["status"] == r.ST_COMPLETED_HEALTH and st.get(free)["status"] == r.ST_INITIAL
    # finished jobs are never claimable again; the remaining lease is intact
    assert [x["id"] for x in st.claim("B", now=1001.0)] == [free]


def test_memory_claim_does_not_scan_live_leases():
    """A claim looks at open jobs and stale holders only (index), not every
    in-progress document of a live worker."""
    st = MemoryJobStore()
    for i in range(2000):
        st.create(_req(i), now=1000.0)
    st.claim("engine", now=1000.0, limit=10_000)
    st.heartbeat("engine", now=1500.0)
    calls = []
    st.create(_req(99999), now=1500.0)
    got = st.claim("w", now=1500.0, only=lambda d: calls.append(d["id"]) or True)
    assert len(got) == 1 and len(calls) == 1


@pytest.mark.parametrize("kind", KINDS)
def test_hyphenated_worker_ids(kind, tmp_path):
    """Worker ids like ``node-m0-rollout``: ES dynamic mapping analyses them into tokens,
    so lease filters must match the exact keyword (the fake analyses strings as ES does)."""
    st = _store(kind, tmp_path)
    ids = [st.create(_req(i), now=1000.0) for i in range(4)]
    a = st.claim("node-m0-rollout", now=1000.0, limit=2)
    st.claim("node-m1-rollout", now=1000.0, limit=2)
    st.heartbeat("node-m0-rollout", now=1100.0)
    # m1 is dead (no heartbeat): its leases are stale at +120 s, m0's are live
    got = st.claim("node-m2-rollout", now=1120.0, max_stuck_s=90.0)
    assert sorted(d["id"] for d in got) == sorted(set(ids) - {d["id"] for d in a})
    # steal_from moves the live holder's leases at once
    st.heartbeat("node-m2-rollout", now=1121.0)
    moved = st.claim("node-m3-rollout", now=1122.0, steal_from={"node-m0-rollout"})
    assert sorted(d["id"] for d in moved) == sorted(d["id"] for d in a)


def test_es_stale_leases_not_crowded_out():
    """More than a search page of live (heartbeat-renewed, so old modified_ts) leases
    must not hide a dead worker's stuck job."""
    st = ElasticJobStore("http://es:9200", transport=httpx.WSGITransport(app=FakeElasticsearch()))
    for i in range(1100):
        st.create(_req(i), now=1000.0)
    st.claim("node-live", now=1000.0, limit=10_000)
    dead = st.create(_req(5000), now=1001.0)
    assert [d["id"] for d in st.claim("node-dead", now=1001.0)] == [dead]
    st.heartbeat("node-live", now=1150.0)
    got = st.claim("node-new", now=1150.0, max_stuck_s=90.0)
    assert [d["id"] for d in got] == [dead]


def test_fake_es_one_mapping_type_per_index():
    es = FakeElasticsearch()
    assert es.handle("PUT", "/idx/document/a", {}, {"x": 1})[0] == 201
    status, body = es.handle("PUT", "/idx/worker/b", {}, {"x": 2})
    assert status == 400 and "more than 1 type" in body["error"]["reason"]
    # the store keeps heartbeats, engine records and jobs each under one type per index
    st = ElasticJobStore("http://es:9200", transport=httpx.WSGITransport(app=es))
    st.create(_req(1), now=1000.0)
    st.heartbeat("node-m0", now=1000.0)
    st.put_meta("cluster_health", {"ok": 1})
    assert st.get_meta("cluster_health") == {"ok": 1}
    assert len(st.claim("node-m0", now=1000.0)) == 1


def test_fake_es_explicit_keyword_mapping_has_no_subfield():
    """On an explicitly keyword-mapped index a `.keyword` filter silently matches
    nothing (as on ES): the store must read the mapping and use the bare field."""
    es = FakeElasticsearch()
    es.handle("PUT", "/documents", {}, {"mappings": {"document": {"properties": {"status": {"type": "keyword"}}}}})
    es.handle("PUT", "/documents/document/a", {}, {"id": "a", "status": "initial"})
    q = {"query": {"bool": {"filter": [{"terms": {"status.keyword": ["initial"]}}]}}, "size": 10}
    assert es.handle("POST", "/documents/document/_search", {}, q)[1]["hits"]["hits"] == []
    q["query"]["bool"]["filter"] = [{"terms": {"status": ["initial"]}}]
    assert len(es.handle("POST", "/documents/document/_search", {}, q)[1]["hits"]["hits"]) == 1
    st = ElasticJobStore("http://es:9200", transport=httpx.WSGITransport(app=es))
    assert st._kw("status") == "status"
    dyn = ElasticJobStore("http://es:9200", transport=httpx.WSGITransport(app=FakeElasticsearch()))
    dyn.create(_req(1), now=1000.0)
    assert dyn._kw("status") == "status.keyword"


def test_es_keyword_detection_reads_typeless_mappings():
    """A typeless (ES 7) mapping response puts `properties` straight under `mappings`;
    the store finds the exact-match field there too."""
    def app(request):
        if request.url.path.endswith("/_mapping"):
            body = {"documents": {"mappings": {"properties": {
                "status": {"type": "keyword"},
                "claimed_by": {"type": "text", "fields": {"keyword": {"type": "keyword"}}}}}}}
            return httpx.Response(200, json=body)
        return httpx.Response(404, json={})
    st = ElasticJobStore("http://es:9200", transport=httpx.MockTransport(app))
    assert st._kw("status") == "status"
    assert st._kw("claimed_by") == "claimed_by.keyword"


def test_es_keyword_negative_answer_is_cached():
    """until the mapping names a field, the fallback is cached for a TTL instead of
    costing one GET /_mapping per search; the mapping is read again after the TTL or once this
    process has written the field."""
    gets = []
    props = {}

    def app(request):
        if request.url.path.endswith("/_mapping"):
            gets.append(1)
            return httpx.Response(200, json={"documents": {"mappings": {"properties": dict(props)}}})
        return httpx.Response(404, json={})
    st = ElasticJobStore("http://es:9200", transport=httpx.MockTransport(app))
    for _ in range(5):
        assert st._kw("claimed_by") == "claimed_by.keyword"
    assert len(gets) == 1
    props["claimed_by"] = {"type": "keyword"}
    st.kw_miss_ttl_s = 0.0            # TTL over: asked again, and the positive answer sticks
    assert st._kw("claimed_by") == "claimed_by"
    assert st._kw("claimed_by") == "claimed_by" and len(gets) == 2
