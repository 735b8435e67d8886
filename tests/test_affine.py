"""Multi-cluster canary on the product path (RC5): cluster A's Prometheus is
scraped only by rank 0, cluster B's only by rank 1.  A canary whose new pods run
in B and whose baseline pods run in A is owned by rank 1; its baseline window
is fetched and decoded by rank 0 and crosses ranks in the node's lockstep
exchange (all_to_all); the job ends completed_unhealth with B's spike."""

import datetime
import json
import os
import subprocess
import sys

import pytest

from foremast_amd.api import rest as r
from foremast_amd.promql import synth
from foremast_amd.promql.fake import FakePrometheus

T0 = 1_700_000_040.0
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HELPER = os.path.join(ROOT, "tests", "helpers", "affine_rank.py")
ENDPOINTS = {"prom-a": "http://prom-a:9090/api/v1/", "prom-b": "http://prom-b:9090/api/v1/"}
M = "http_server_requests_error_5xx"
# app -> (cluster of the new pods + history, cluster of the baseline pods, spike)
APPS = {"shop": ("prom-b", "prom-a", True), "cart": ("prom-b", "prom-a", False), "inv": ("prom-a", "prom-b", False)}


def clusters(clock):
    proms = {h: FakePrometheus(clock=clock) for h in ENDPOINTS}
    for i, (app, (cur, base, spike)) in enumerate(APPS.items()):
        lvl = 0.3 + 0.1 * i
        proms[cur].add("namespace_app_per_pod:" + M, {"namespace": "ns", "app": app},
                       synth.error_rate(base=lvl, spread=0.05, seed=i))
        for k in range(2):
            gen = synth.error_rate(base=lvl, spread=0.05, seed=100 + 10 * i + k)
            if spike:
                gen = synth.step_change(gen, at=T0 + 120, factor=0.0, add=40.0)
            proms[cur].add("namespace_pod:" + M, {"namespace": "ns", "pod": f"{app}-v2-{k}"}, gen)
        for k in range(3):
            proms[base].add("namespace_pod:" + M, {"namespace": "ns", "pod": f"{app}-v1-{k}"},
                            synth.error_rate(base=lvl, spread=0.05, seed=200 + 10 * i + k))
    return proms


def request(app):
    from foremast_amd.utils.timeutil import format_rfc3339
    cur, base, _ = APPS[app]

    def q(ep, query, start, end):
        return {"dataSourceType": "prometheus",
                "parameters": {"endpoint": ENDPOINTS[ep], "query": query, "start": int(start), "end": int(end),
                               "step": 60}}
    pods = "|".join(f"{app}-v2-{k}" for k in range(2))
    old = "|".join(f"{app}-v1-{k}" for k in range(3))
    return {"appName": app, "startTime": format_rfc3339(T0), "endTime": format_rfc3339(T0 + 600),
            "strategy": "canary", "metrics": {
                "current": {"error5xx": q(cur, f'namespace_pod:{M}{{namespace="ns",pod=~"{pods}"}}', T0 + 60, T0 + 660)},
                "baseline": {"error5xx": q(base, f'namespace_pod:{M}{{namespace="ns",pod=~"{old}"}}', T0 - 600, T0)},
                "historical": {"error5xx": q(cur, f'namespace_app_per_pod:{M}{{namespace="ns",app="{app}"}}',
                                             T0 - 7 * 86400, T0)}}}


@pytest.mark.slow
@pytest.mark.parametrize("fail_beat", [None, "1"])
def test_multi_cluster_canary_crosses_ranks(tmp_path, fail_beat):
    """``fail_beat``: rank 1's store heartbeat raises on two ticks; the lockstep exchange
    must still run on that rank (else the peers' collectives desynchronise) and the
    verdicts must not change."""
    import torch.distributed as dist
    from foremast_amd.service import app as svc
    from foremast_amd.store.jobstore import SqliteJobStore
    db = str(tmp_path / "jobs.db")
    store = SqliteJobStore(db)
    ids = {a: svc.register(store, request(a))[1]["jobId"] for a in APPS}
    kv = dist.TCPStore("127.0.0.1", 0, is_master=True, wait_for_workers=False, timeout=datetime.timedelta(seconds=60))
    env = dict(os.environ, OMP_NUM_THREADS="1", CUDA_VISIBLE_DEVICES="",
               FOREMAST_CLUSTER_AFFINITY=f"{ENDPOINTS['prom-a']}=0,{ENDPOINTS['prom-b']}=1")
    if fail_beat is not None:
        env["AFFINE_FAIL_BEAT"] = fail_beat
    outs = [tmp_path / f"rank{i}.jsonl" for i in range(2)]
    procs = [subprocess.Popen([sys.executable, HELPER, str(kv.port), str(i), db, str(outs[i])], env=env, cwd=ROOT,
                              stderr=subprocess.PIPE, text=True) for i in range(2)]
    errs = [p.communicate(timeout=300)[1] for p in procs]
    assert all(p.returncode == 0 for p in procs), "\n".join(e[-3000:] for e in errs)
    lines = [[json.loads(x) for x in o.read_text().splitlines()] for o in outs]
    first = [ls[0] for ls in lines]
    assert first[1]["jobs"] == ["cart", "shop"] and first[0]["jobs"] == ["inv"]   # owned by the new pods' cluster
    # the baseline (3 pods x 11 points) came from the other rank's cluster
    assert first[1]["base_valid"] == {"cart": 33, "shop": 33} and first[0]["base_valid"] == {"inv": 33}
    assert all(ls[-1]["values_moved"] > 0 for ls in lines)
    assert lines[0][-1]["exchanges"] == lines[1][-1]["exchanges"] > 0  # the ranks stayed in lockstep
    assert first[0]["scrapes"]["prom-b"] == 0 and first[1]["scrapes"]["prom-a"] == 0  # cluster-affine scraping
    st = {a: store.get(j) for a, j in ids.items()}
    assert st["shop"]["status"] == r.ST_COMPLETED_UNHEALTH, st["shop"]
    vals = json.loads(st["shop"]["anomalyInfo"])["error5xx"]["values"]
    assert vals[1] > 30
    assert st["cart"]["status"] == r.ST_COMPLETED_HEALTH and st["inv"]["status"] == r.ST_COMPLETED_HEALTH


def test_request_lists_larger_than_a_store_value_are_chunked():
    """A burst of admissions publishes more than the store's 8 MiB value cap: the
    requests go in chunks and every peer reassembles them (two ranks sharing one store)."""
    import threading

    import torch
    import torch.distributed as dist
    from foremast_amd.parallel.affine import CHUNK, ClusterRouter
    kv = dist.HashStore()
    reqs = {r: [(("http://prom-%d/" % r, "namespace_pod:m"), 1.7e9, 11,
                 [("ns%d" % (i % 7), "app%d-v1-%d-5b6c7d8e9f" % (i, r)) for i in range(j * 500, (j + 1) * 500)])
                for j in range(2 * CHUNK // 20000)] for r in range(2)}
    got = {}

    def rank(r):
        rt = ClusterRouter(lambda ep, w: 0, torch.device("cpu"), kv=kv)
        got[r] = rt._gather_requests(reqs[r], 2, r)
    ts = [threading.Thread(target=rank, args=(r,)) for r in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(60)
    assert len(json_size := str(reqs[0])) > CHUNK and json_size
    for r in range(2):
        assert [(q[0], q[1], q[2], list(q[3])) for q in got[r][1 - r]] == \
            [(q[0], q[1], q[2], list(q[3])) for q in reqs[1 - r]]
