"""Node health exchange under churn: N ranks equal one rank, every tick.

Every tick apps start and finish (a sliding window of the app pool; finished
apps' table indices are reused), each rank holds its apps in two engines (some
apps in both: the merged roster's reference counts), and the node brain runs
the deployed exchange — ElasticWorld.run_tick, one all-gather of counters,
roster DELTAS through the generation's store (``parallel/cluster.py``).  The
node table (every app's counters and the anomalous apps) must equal the 1-rank
table and the analytic one on every tick, on every rank, at 2, 4 and 8 gloo
ranks; the roster bytes per tick must follow the changes, not the roster size.
Reference: brains scale out and aggregate health across clusters
(``/root/reference/docs/guides/design.md:37-41``, ``/root/reference/README.md:27``).
"""

import datetime
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from foremast_amd.brain.node import owner_of

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HELPER = os.path.join(ROOT, "tests", "helpers", "roster_rank.py")
sys.path.insert(0, os.path.join(ROOT, "tests", "helpers"))
from roster_rank import counts_of, engines_of, live_apps  # noqa: E402

TICKS, PER_TICK, SPAN = 24, 12, 180


def run(tmp_path, n):
    import torch.distributed as dist
    kv = dist.TCPStore("127.0.0.1", 0, is_master=True, wait_for_workers=False, timeout=datetime.timedelta(seconds=90))
    procs, outs = [], []
    for i in range(n):
        out = tmp_path / f"roster_n{n}_r{i}.jsonl"
        env = dict(os.environ, OMP_NUM_THREADS="1", CUDA_VISIBLE_DEVICES="", GLOO_SOCKET_IFNAME="lo")
        procs.append(subprocess.Popen([sys.executable, HELPER, str(kv.port), str(i), str(n), str(TICKS),
                                       str(PER_TICK), str(SPAN), str(out)], env=env, cwd=ROOT,
                                      stderr=subprocess.PIPE, text=True))
        outs.append(out)
    try:
        for p in procs:
            _, err = p.communicate(timeout=300)
            assert p.returncode == 0, err[-4000:]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return [[json.loads(x) for x in o.read_text().splitlines()] for o in outs]


def expected(k, n):
    apps = {}
    for a in live_apps(k, PER_TICK, SPAN):
        c = np.sum([counts_of(a, k, e) for e in engines_of(a)], axis=0).tolist()
        apps[f"ns/app{a}"] = (c, owner_of("ns", f"app{a}", n))
    return apps


@pytest.mark.slow
def test_churning_roster_n_ranks_equal_one_rank(tmp_path):
    ref = run(tmp_path, 1)[0]
    for k, line in enumerate(ref):
        want = expected(k, 1)
        assert {a: v for a, v in line["apps"].items()} == {a: c for a, (c, _) in want.items()}, k
    rec = {}
    for n in (2, 4, 8):
        lines = run(tmp_path, n)
        for rank_lines in lines:
            assert len(rank_lines) == TICKS
            for k, (line, r1) in enumerate(zip(rank_lines, ref)):
                assert line["apps"] == r1["apps"], (n, k)
                assert line["anomalous"] == r1["anomalous"], (n, k)
                assert line["generation"] == 0
        # bytes through the store per tick follow the changes: after the first full rosters,
        # each rank publishes ~(2 x PER_TICK / n) changes and reads the other ranks' deltas
        steady = [ln["roster_bytes"] for ln in lines[0][2:]]
        full = max(ln["roster_bytes"] for ln in lines[0][:1])
        assert np.median(steady) < 0.5 * full or full < 2000, (n, steady, full)
        ms = [ln["exchange_ms"] for ls in lines for ln in ls[2:]]
        own = [ln["phases"]["publish"] + ln["phases"]["rosters"] + ln["phases"]["table"] for ls in lines for ln in ls[2:]]
        rec[n] = {"exchange_ms_p50": float(np.percentile(ms, 50)), "exchange_ms_p90": float(np.percentile(ms, 90)),
                  "roster_and_table_ms_p50": float(np.percentile(own, 50)),
                  "roster_bytes_p50": float(np.median(steady)), "first_tick_bytes": full}
    (tmp_path / "exchange_record.json").write_text(json.dumps(rec))
    print("exchange record", json.dumps(rec))


def test_node_roster_pass_and_merged_modes_match_the_engines():
    """NodeRoster over two engines whose apps come and go (indices reused), passing
    through one engine's table while the other is empty and merging when both hold
    apps: every tick the node table (name -> summed counters) equals the engines',
    and a peer replaying the node's change log (resets: a full copy) holds the same
    roster -- what ClusterHealth's deltas rely on."""
    import random
    import torch
    from foremast_amd.parallel.roster import ChangeLog, NodeRoster

    class Eng:
        def __init__(self):
            self.names, self.index, self.free, self.log = [], {}, [], ChangeLog()

        def set(self, apps):
            for nm in [n for n in self.index if n not in apps]:
                i = self.index.pop(nm)
                self.names[i] = None
                self.free.append(i)
                self.log.note(i, None)
            for nm in apps:
                if nm not in self.index:
                    i = self.free.pop() if self.free else len(self.names)
                    if i == len(self.names):
                        self.names.append(nm)
                    else:
                        self.names[i] = nm
                    self.index[nm] = i
                    self.log.note(i, nm)

    rng = random.Random(5)
    eng = [Eng(), Eng()]
    nr = NodeRoster(2, "cpu")
    mirror = []
    modes = set()
    for tick in range(60):
        phase = (tick // 12) % 3        # 0: engine 0 only, 1: both, 2: engine 1 only
        pool = [("ns", f"a{i}") for i in range(40)]
        for k, e in enumerate(eng):
            on = (phase == 0 and k == 0) or phase == 1 or (phase == 2 and k == 1)
            e.set(set(rng.sample(pool, rng.randint(3, 25))) if on else set())
        tables = [torch.tensor([[rng.randint(0, 1), rng.randint(1, 4)] if n else [0, 0] for n in e.names],
                               dtype=torch.int32).reshape(-1, 2) for e in eng]
        engines = []
        for e in eng:
            reset, items = e.log.drain()
            engines.append((reset, items, (lambda e=e: e.names), len(e.index)))
        nr.update(engines)
        modes.add(nr.mode[0])
        got = {n: nr.counts(tables)[i].tolist() for i, n in enumerate(nr.names) if n}
        want = {}
        for e, t in zip(eng, tables):
            for n, i in e.index.items():
                c = want.setdefault(n, [0, 0])
                c[0] += int(t[i, 0])
                c[1] += int(t[i, 1])
        assert got == want, tick
        reset, items = nr.log.drain()
        if reset:
            mirror = list(nr.names)
        for i, n in items:
            mirror.extend([None] * (i + 1 - len(mirror)))
            mirror[i] = n
        assert [n for n in mirror if n] == [n for n in nr.names if n] and \
            {i: n for i, n in enumerate(mirror) if n} == {i: n for i, n in enumerate(nr.names) if n}, tick
    assert modes == {"pass", "merged"}


def test_pass_through_roster_is_a_snapshot_of_the_exchange():
    """in pass-through mode the node's names are the rank's own list as of the
    exchange: an engine that frees an app and admits another at the same index AFTER the
    exchange (intake runs later in the tick) must not rename the published counters."""
    import torch
    from foremast_amd.parallel.roster import ChangeLog, NodeRoster
    names, log = [("ns", "a"), ("ns", "b")], ChangeLog()
    log.note(0, names[0])
    log.note(1, names[1])
    nr = NodeRoster(1, "cpu")
    reset, items = log.drain()
    nr.update([(reset, items, lambda: names, 2)])
    table = torch.tensor([[1, 5], [0, 5]], dtype=torch.int32)
    before = list(nr.names)
    # intake after the exchange: "a" finishes, "c" is admitted into its index
    names[0] = None
    log.note(0, None)
    names[0] = ("ns", "c")
    log.note(0, ("ns", "c"))
    assert nr.names == before and nr.names[0] == ("ns", "a")
    assert nr.counts([table])[0].tolist() == [1, 5]
    # the next exchange applies the changes (O(changes), no full copy)
    reset, items = log.drain()
    assert not reset
    assert nr.update([(reset, items, lambda: names, 2)])
    assert nr.names == [("ns", "c"), ("ns", "b")] and nr.names is not names
