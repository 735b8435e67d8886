import asyncio
import json

import httpx
import numpy as np
import pytest

from foremast_amd.ingest import native
from foremast_amd.promql import synth
from foremast_amd.promql.client import PromClient
from foremast_amd.promql.fake import FakePrometheus
from foremast_amd.promql.selector import SelectorError, parse_selector


def test_selector_matching():
    s = parse_selector('namespace_pod:http_server_requests_error_5xx{namespace="ns",pod=~"a-1|b-2"}')
    assert s.name == "namespace_pod:http_server_requests_error_5xx"
    base = {"__name__": s.name, "namespace": "ns"}
    assert s.matches(dict(base, pod="a-1"))
    assert not s.matches(dict(base, pod="a-10"))  # anchored regex
    assert not s.matches(dict(base, pod="c"))
    s2 = parse_selector('m{app!="x",pod!~"z.*"}')
    assert s2.matches({"__name__": "m", "app": "y", "pod": "a"})
    with pytest.raises(SelectorError):
        parse_selector("sum(rate(x[1m]))")


BODY = (b'{"status":"success","data":{"resultType":"matrix","result":['
        b'{"metric":{"__name__":"m","pod":"a"},"values":[[1700000000,"1.5"],[1700000060,"NaN"],[1700000120,"2"]]},'
        b'{"metric":{},"values":[]},'
        b'{"metric":{"pod":"b\\"q"},"values":[[1700000060.5,"+Inf"],[1700000180,"-3e-2"]]}]}}')


def test_native_parser_matches_json():
    out = native.parse_matrix(BODY)
    ref = native._parse_py(BODY)
    assert len(out) == len(ref) == 3
    for (l1, t1, v1), (l2, t2, v2) in zip(out, ref):
        assert l1 == l2
        np.testing.assert_array_equal(t1, t2)
        np.testing.assert_array_equal(v1, v2)
    assert out[2][0]["pod"] == 'b"q'


def test_native_dense_scatter():
    dense = np.full((4, 5), np.nan, dtype=np.float32)
    n, dropped = native.parse_dense(BODY, 1700000000, 60, 5, dense, row0=1)
    assert n == 3
    assert dropped == 1  # the off-grid 1700000060.5 sample
    assert dense[1, 0] == 1.5 and np.isnan(dense[1, 1]) and dense[1, 2] == 2.0
    assert dense[3, 3] == pytest.approx(-0.03)


def test_parser_errors():
    with pytest.raises(native.ParseError):
        native.parse_matrix(b'{"status":"error","errorType":"bad_data","error":"x"}')
    with pytest.raises(native.ParseError):
        native.parse_matrix(b'{"status":"success","data":{"result":[{"metric":{},"values":[[1,}]}}')


def test_fake_prometheus_and_client_roundtrip():
    prom = FakePrometheus(clock=lambda: 1_700_100_000)
    prom.add("namespace_pod:lat", {"namespace": "ns", "pod": "p1"}, synth.seasonal(level=10, amp=1, noise=0.1))
    prom.add("namespace_pod:lat", {"namespace": "ns", "pod": "p2"}, synth.seasonal(level=12, amp=1, noise=0.1))
    prom.add("namespace_pod:lat", {"namespace": "other", "pod": "p1"}, synth.seasonal())
    transport = httpx.ASGITransport(app=prom.asgi_app())
    client = PromClient(transport=transport)
    url = ("http://prom:9090/api/v1/query_range?query=" + "namespace_pod%3Alat%7Bnamespace%3D%22ns%22%2Cpod%3D~%22p1%7Cp2%22%7D"
           + "&start=1700000000&end=1700003540&step=60")
    res = asyncio.run(client.fetch_many([url]))[0]
    assert len(res) == 2
    assert all(len(s.ts) == 60 for s in res)
    assert {s.labels["pod"] for s in res} == {"p1", "p2"}
    # late data: nothing newer than now - lag
    prom.faults.lag_seconds = 1_700_100_000 - 1_700_001_000
    res = asyncio.run(client.fetch_many([url]))[0]
    assert all(s.ts.max() <= 1_700_001_000 for s in res)


def test_error_rate_spikes():
    f = synth.error_rate(spikes=[600.0, 1800.0])
    v = f(np.arange(0, 3600, 60.0))
    assert v[10] > 30 and v[30] > 30
    assert np.all(v[[0, 5, 20, 40]] < 2)


def test_tick_decoder_round_trips_pod_bodies():
    """Bodies rendered per (app, pod) decode, in parallel and double-buffered,
    into exactly the float32 block they were rendered from."""
    import torch
    from foremast_amd.ingest import native
    from foremast_amd.ingest.tickdecode import TickDecoder, pod_matrix_body
    rng = np.random.default_rng(0)
    n_app, P = 300, 4
    vals = rng.normal(50, 10, (2, n_app, 2 * P)).astype(np.float32)
    vals[0, 7, 3] = np.nan
    labels, rows = [], []
    for kind in range(2):
        labels.append([f'"app":"a{a}","pod":"a{a}-{kind}{p}"' for a in range(n_app) for p in range(P)])
        rows.append((np.arange(n_app)[:, None] * 2 * P + kind * P + np.arange(P)[None, :]).reshape(-1))
    bodies = [[pod_matrix_body("m", labels[kind], 600 * (k + 1), vals[k, :, kind * P:(kind + 1) * P].reshape(-1))
               for kind in range(2)] for k in range(2)]
    tables = [native.KeyTable.from_hashes(native.series_keys(b, "app", "pod"), r, "app", "pod")
              for b, r in zip(bodies[0], rows)]
    dec = TickDecoder(tables, n_app * 2 * P, 1, pinned=False, threads=2)
    futs = [dec.submit(bodies[k], 600 * (k + 1), 60.0) for k in range(2)]
    for k, f in enumerate(futs):
        block, stats = f.result()
        assert [s[2] for s in stats] == [0, 0]  # every series matched a row
        np.testing.assert_array_equal(block.view(n_app, 2 * P).numpy(), vals[k])
    dec.close()


def test_bench_prom_ingest_matches_pinned_ingest():
    """bench --ingest prom (JSON bodies decoded inside the tick) scores exactly
    what the pinned-arrival path scores."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = []
    for mode in ("pinned", "prom"):
        out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--cpu", "--steps", "2", "--warmup",
                              "1", "--ingest", mode, "--anomaly-frac", "0.05"], capture_output=True, text=True,
                             timeout=600, env=dict(os.environ, OMP_NUM_THREADS="2"))
        assert out.returncode == 0, out.stderr[-2000:]
        res.append(json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][0]))
    assert res[0]["health"] == res[1]["health"] and res[0]["detection"] == res[1]["detection"]
    assert res[1]["config"]["ingest"] == "prom" and res[1]["config"]["ingest_bytes_per_tick"] > 0


def test_decode_bodies_matches_per_body_decode_and_learns_layout():
    """A history load's bodies (time chunks x app groups, each with its own grid
    start and column offset, one key table per family) decode in ONE threaded
    native call into exactly what per-body keyed decodes produce — including a
    malformed body in the middle (reported; its complete series and all other
    bodies still decoded) and a
    second pass over the same bodies, which runs on the learned layout."""
    from foremast_amd.ingest import native
    rng = np.random.default_rng(3)
    n_app, chunk, n_chunk, step = 120, 30, 4, 60.0
    t0 = 1_700_000_000.0
    vals = rng.normal(20, 5, (n_app, chunk * n_chunk)).astype(np.float32)
    vals[5, 17] = np.nan
    keys = [(f"ns{a % 3}", f"app{a}") for a in range(n_app)]
    table = native.KeyTable([(k, i) for i, k in enumerate(keys)])

    def body(apps, c):
        items = []
        for a in apps:
            pts = ",".join(f'[{int(t0 + (c * chunk + i) * step)},"{float(vals[a, c * chunk + i]):.9g}"]'
                           for i in range(chunk))
            items.append(f'{{"metric":{{"__name__":"m","namespace":"{keys[a][0]}","app":"{keys[a][1]}"}},'
                         f'"values":[{pts}]}}')
        return ('{"status":"success","data":{"resultType":"matrix","result":[' + ",".join(items) + "]}}").encode()

    groups = [range(0, 50), range(50, 120)]
    bodies, starts, cols = [], [], []
    for c in range(n_chunk):
        for g in groups:
            bodies.append(body(g, c))
            starts.append(t0 + c * chunk * step)
            cols.append(c * chunk)
    bad = len(bodies) // 2
    bodies[bad] = bodies[bad][: len(bodies[bad]) // 2]  # truncated response
    ref = np.full((n_app, chunk * n_chunk), np.nan, dtype=np.float32)
    for j, (b, st, c0) in enumerate(zip(bodies, starts, cols)):
        try:  # the truncated body writes its complete series, then fails (both decoders)
            native.parse_dense_keyed(b, st, step, chunk, ref, table, col0=c0)
        except native.ParseError:
            assert j == bad
    for _ in range(2):
        out = np.full_like(ref, np.nan)
        stats = native.decode_bodies(bodies, [table] * len(bodies), starts, step, [chunk] * len(bodies), cols, out,
                                     threads=3)
        assert stats[bad][0] < 0
        assert all(s[0] == len(groups[j % 2]) and s[2] == 0 for j, s in enumerate(stats) if j != bad)
        np.testing.assert_array_equal(out, ref)


def test_family_bodies_share_one_index_layout():
    """One tick's family bodies (same pods, label objects that differ only in the
    leading ``__name__``) through ONE shared pod index: each pass decodes exactly,
    including after the pod order of one family changes, a pod leaves, a metric name
    carries an escape, and with ``__name__`` as a key label (then no name is skipped)."""
    from foremast_amd.ingest import native
    rng = np.random.default_rng(5)
    n, F = 300, 4
    pods = [(f"ns{i % 7}", f"app{i // 3}-v2-{i % 3}-7d9f") for i in range(n)]
    ix = native.LiveKeyIndex("namespace", "pod")
    ix.set(native.key_hashes([a for a, _ in pods], [b for _, b in pods]), np.arange(n))

    def body(name, order, vals):
        items = [f'{{"metric":{{"__name__":"{name}","namespace":"{pods[i][0]}","pod":"{pods[i][1]}"}},'
                 f'"values":[[600000,"{float(vals[i]):.9g}"]]}}' for i in order]
        return ('{"status":"success","data":{"resultType":"matrix","result":[' + ",".join(items) + "]}}").encode()

    names = [f"namespace_pod:m{f}" for f in range(F - 1)] + ['namespace_pod:m\\"q']
    for rnd in range(4):
        vals = rng.normal(50, 9, (F, n)).astype(np.float32)
        orders = [list(range(n)) for _ in range(F)]
        if rnd == 2:
            orders[1] = list(rng.permutation(n))   # one family lists its pods in another order
            orders[3] = orders[3][:100] + orders[3][101:]  # a pod missing from one family
        bodies = [body(names[f], orders[f], vals[f]) for f in range(F)]
        out = np.full((n, F), np.nan, dtype=np.float32)
        stats = native.decode_bodies(bodies, [ix] * F, [600000.0] * F, 60.0, [1] * F, list(range(F)), out, threads=3)
        assert [s[0] for s in stats] == [len(o) for o in orders] and all(s[2] == 0 for s in stats)
        ref = vals.T.copy()
        if rnd == 2:
            ref[100, 3] = np.nan
        np.testing.assert_array_equal(out, ref)
    # keyed on __name__ itself: the metric name is part of the key and is never skipped
    t = native.KeyTable([((names[f], pods[0][1]), f) for f in range(F)], "__name__", "pod")
    for _ in range(2):
        out = np.full((F, 1), np.nan, dtype=np.float32)
        one = np.full(n, 7.0, dtype=np.float32)
        for f in range(F):
            one[0] = 10 + f
            native.decode_bodies([body(names[f], [0], one)], [t], [600000.0], 60.0, [1], [0], out, threads=1)
        np.testing.assert_array_equal(out[:, 0], 10 + np.arange(F, dtype=np.float32))


def test_keyed_decoder_number_shapes_match_python_float():
    """The keyed decoder's number paths — the 8-digits-at-a-time decimal path, the
    per-digit exact path, ``from_chars``, the special values — and the per-ordinal
    timestamp cache (compact and spaced samples, repeated and fresh timestamp text)
    give exactly ``float32(float(text))`` for every sample shape."""
    from foremast_amd.ingest import native
    texts = ["12", "-3.5", "0.000123", "5.", ".5", "-0", "00012.50", "1234567890123456", "12345678.12345678",
             "1e5", "-2.5E-3", "9007199254740993", "NaN", "+Inf", "-Inf", "49.6630936", "-0.000000001",
             "123456789.5", "7", "99999999.99999999"]
    t0, step, T = 1_700_000_000, 60.0, len(texts)
    keys = [("ns", f"app{a}") for a in range(6)]
    table = native.KeyTable([(k, i) for i, k in enumerate(keys)])
    items, want = [], np.full((len(keys), T), np.nan, dtype=np.float32)
    for a in range(len(keys)):
        rot = texts[a:] + texts[:a]
        ts_txt = [str(t0 + int(step) * j) if a % 3 else f"{t0 + int(step) * j}.000" for j in range(T)]
        if a == 4:
            pts = ", ".join(f'[ {ts_txt[j]} , "{rot[j]}" ]' for j in range(T))
        else:
            pts = ",".join(f'[{ts_txt[j]},"{rot[j]}"]' for j in range(T))
        items.append(f'{{"metric":{{"namespace":"ns","app":"app{a}"}},"values":[{pts}]}}')
        want[a] = [np.float32(float(x)) for x in rot]
    body = ('{"status":"success","data":{"resultType":"matrix","result":[' + ",".join(items) + "]}}").encode()
    for _ in range(2):  # the second pass runs on the learned layout
        out = np.full_like(want, np.nan)
        assert native.parse_dense_keyed(body, t0, step, T, out, table) == (len(keys), 0, 0)
        np.testing.assert_array_equal(out, want)
        out = np.full_like(want, np.nan)
        stats = native.decode_bodies([body], [table], [t0], step, [T], [0], out, threads=2)
        assert stats == [(len(keys), 0, 0)]
        np.testing.assert_array_equal(out, want)
    for bad in ("1.2.3", "12a", "-", "."):
        b = body.replace(b'"49.6630936"', f'"{bad}"'.encode(), 1)
        with pytest.raises(native.ParseError):
            native.parse_dense_keyed(b, t0, step, T, np.full_like(want, np.nan), table)
