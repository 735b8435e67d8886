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
    return ElasticJobStore("http://es:9200", transport=httpx.WSGITransport(app=FakeElasticsearch()))


def _req(i):
    return r.DocumentRequest(app_name=f"app{i}", start_time="2023-11-14T22:13:20Z", end_time="2023-11-14T22:23:20Z",
                             current_config=f"m== http://p/api/v1/query_range?query=x{i}", strategy="canary")


@pytest.mark.parametrize("kind", ["memory", "sqlite", "es"])
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


@pytest.mark.parametrize("kind", ["memory", "sqlite", "es"])
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
