"""Continuous monitoring on the streaming GPU engine.

Continuous jobs (``strategy: continuous`` — barrelman's ``monitorContinuously``,
``Barrelman.go:176-203``) ask the same question every minute for as long as
the job runs.  Instead of refetching and refitting each job independently
(what :class:`~foremast_amd.brain.worker.BrainWorker` does for one-shot
canary/rollout jobs), the :class:`StreamingMonitor` keeps every continuous
series resident in one :class:`~foremast_amd.brain.engine.StreamingShard`:

* rows: one per (endpoint, metric, namespace, app) series.  Rows are stable
  while a series is live; a new job's series take free rows (the shard grows
  by doubling when full) and only THEIR history is fetched, a finished job's
  rows are cleared and freed — no full rebuild on membership changes;
* history: 7 days at the query step, fetched in chunks that stay far below
  Prometheus' ``--query.max-samples`` (≤ ``history_chunk_points`` per query in
  time and ≤ ``apps_per_query`` apps per selector, ``app=~"a|b|…"``), decoded
  by the native keyed parser straight into a pinned staging block (each series
  lands in its row, no per-series Python) and copied H2D in one transfer;
* every tick: one short range query per metric family for the newest points of
  all series → keyed decode into a pinned ``[rows, k]`` block → H2D → tick
  ingest kernel per point → one fused scoring launch for all series → per-job
  verdicts;
* jobs: leased from the job store with a strategy filter (the one-shot worker
  skips them) and an optional ownership filter (``owns``: the node brain
  shards apps over GPU ranks, ``brain/node.py``); any anomalous series
  finishes its job ``completed_unhealth`` with the anomalous points; past
  ``endTime`` a job finishes ``completed_health``; band gauges are exported
  for the UI; per-app counters feed the node health table.
"""

from __future__ import annotations

import asyncio
import json
import logging
import re
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Set, Tuple
from urllib.parse import quote

import numpy as np
import torch

from ..parallel.roster import ChangeLog
from ..api import rest as r
from ..ingest import native
from ..promql.client import PromClient
from ..promql.selector import SelectorError, parse_selector
from ..service import urls
from ..store.jobstore import JobStore
from ..utils.config import BrainConfig
from ..utils.metrics import BrainMetrics
from ..utils.timeutil import TimeFormatError, parse_rfc3339
from .engine import ShardSpec, StreamingShard
from .resident import fetch_decode

log = logging.getLogger("foremast.streaming")

STRATEGY_CONTINUOUS = "continuous"
Key = Tuple[str, str, str, str]  # (endpoint, metric, namespace, app)


def is_continuous(doc) -> bool:
    return (doc.get("strategy") or "").lower() == STRATEGY_CONTINUOUS


CALLER_SPLIT = ("namespace_pod_caller:", "namespace_app_caller:", "namespace_app_caller_per_pod:",
                "namespace_pod_uri:", "namespace_app_uri:", "namespace_app_uri_per_pod:")


def is_streamable(doc) -> bool:
    """Continuous jobs whose series are one per (namespace, app): the resident
    GPU shard's keying.  Downstream (per-caller) and API-level (per-uri) metrics
    split an app into one series per caller / path, so such jobs stay with the
    batch worker (brain/worker.py)."""
    return is_continuous(doc) and not any(k[1].startswith(CALLER_SPLIT) for k in series_of(doc).values())


def series_of(doc) -> Dict[str, Key]:
    """alias → series key of a job's historical queries."""
    out = {}
    for alias, url in urls.parse_config(doc.get("historicalConfig", "")).items():
        try:
            p = urls.parse_prometheus_url(url)
            sel = parse_selector(str(p["query"]))
        except (urls.ConfigError, SelectorError):
            continue
        lab = {k: v for k, op, v in sel.matchers if op == "="}
        endpoint = url.split("query_range?")[0]
        out[alias] = (endpoint, sel.name, lab.get("namespace", ""), lab.get("app", ""))
    return out


def app_of(doc) -> Tuple[str, str]:
    """(namespace, app) a job monitors: the first historical selector's labels,
    else the job's appName."""
    for key in series_of(doc).values():
        if key[3]:
            return key[2], key[3]
    return "", doc.get("appName", "")


_RE2_SPECIAL = re.compile(r"([\\.^$|?*+()\[\]{}])")


def _re_alt(values) -> str:
    """RE2 alternation of literal label values, escaped for a PromQL string."""
    return "|".join(_RE2_SPECIAL.sub(r"\\\\\1", v) for v in sorted(values))


@dataclass
class StreamJob:
    doc: Dict
    end_ts: float
    series: Dict[str, Key] = field(default_factory=dict)  # alias -> series key


class StreamingMonitor:
    def __init__(self, store: JobStore, cfg: Optional[BrainConfig] = None, prom: Optional[PromClient] = None,
                 device=None, worker_id: str = "stream-0", metrics: Optional[BrainMetrics] = None,
                 ring_len: int = 10080, step: float = 60.0, window: int = 10, clock=time.time,
                 owns: Optional[Callable[[Dict], bool]] = None, history_chunk_points: int = 1440,
                 apps_per_query: int = 256, min_capacity: int = 64, decode_threads: Optional[int] = None) -> None:
        self.store = store
        self.cfg = cfg or BrainConfig.from_env()
        self.prom = prom or PromClient()
        self.device = torch.device(device) if device is not None else (
            torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu"))
        self.worker_id = worker_id
        self.metrics = metrics or BrainMetrics()
        self.R, self.step, self.W = ring_len, step, window
        self.clock = clock
        self.owns = owns
        self.exclude: Optional[Callable[[Dict], bool]] = None  # jobs another resident engine serves (LSTM)
        self.chunk_pts = max(1, int(history_chunk_points))
        self.apps_per_query = max(1, int(apps_per_query))
        self.decode_threads = max(1, int(decode_threads or native.default_threads()))  # native threads decoding the responses
        self.min_capacity = min_capacity
        self.jobs: Dict[str, StreamJob] = {}
        self.keys: List[Optional[Key]] = []          # row -> key (None: free row)
        self.rows: Dict[Key, int] = {}
        self.pending: Set[Key] = set()               # live keys whose history is not loaded yet
        self.apps: Dict[Tuple[str, str], int] = {}   # (namespace, app) -> app index (node health table)
        self.roster_version = 0
        self.roster_log = ChangeLog()
        self.shard: Optional[StreamingShard] = None
        self.t_last: float = 0.0
        self.ticks = 0
        self.history_queries = 0
        self._table: Optional[Dict[Tuple[str, str], native.KeyTable]] = None

    # ------------------------------------------------------------------ membership
    def sync(self, steal_from=None) -> int:
        """Lease new continuous jobs (that this rank owns); returns how many were added."""
        now = self.clock()

        def only(d):
            return (is_streamable(d) and (self.owns is None or self.owns(d))
                    and (self.exclude is None or not self.exclude(d)))
        docs = self.store.claim(self.worker_id, now=now, max_stuck_s=self.cfg.max_stuck_seconds, limit=10_000,
                                only=only, steal_from=steal_from)
        for d in docs:
            try:
                end_ts = parse_rfc3339(d.get("endTime", "")).timestamp()
            except TimeFormatError:
                end_ts = float("inf")
            job = StreamJob(doc=d, end_ts=end_ts, series=series_of(d))
            for key in job.series.values():
                if key not in self.rows:
                    self.pending.add(key)
            self.jobs[d["id"]] = job
        return len(docs)

    def release(self, pred: Callable[[Dict], bool]) -> int:
        """Hand back the leases of jobs matching ``pred`` (re-sharding: another
        rank owns their app now); their series are freed at the next tick."""
        n = 0
        for jid, job in list(self.jobs.items()):
            if pred(job.doc):
                self.store.update(jid, {"status": r.ST_REPROGRESS, "claimed_by": "", "not_before": 0.0},
                                  expect_claimed_by=self.worker_id)
                del self.jobs[jid]
                n += 1
        return n

    def live_keys(self) -> Set[Key]:
        return {k for j in self.jobs.values() for k in j.series.values()}

    @property
    def n_live(self) -> int:
        return len(self.rows)

    # ------------------------------------------------------------------ rows
    def _new_shard(self, capacity: int) -> StreamingShard:
        season = max(2, int(round(86400.0 / self.step)))
        algo = self.cfg.algorithm if self.cfg.algorithm in ("holt_winters", "exponential_smoothing",
                                                            "double_exponential_smoothing", "moving_average",
                                                            "moving_average_all", "seasonal_decompose") \
            else "moving_average_all"
        if algo == "holt_winters" and self.R < 2 * season:
            algo = "double_exponential_smoothing"
        if algo == "seasonal_decompose" and self.R < 2 * season + 1:
            algo = "moving_average_all"
        dev = self.device
        spec = ShardSpec(n_series=capacity, ring_len=self.R, season=season, pods=1, window=self.W, algorithm=algo,
                         pairwise="NONE", dtype=torch.bfloat16 if dev.type == "cuda" else torch.float32,
                         n_apps=max(1, len(self.apps)))
        sh = StreamingShard(spec, self.cfg, dev)
        sh.hist.state.head, sh.hist.state.length = 0, self.R   # rows start all-NaN (free)
        sh.cur.ticks = self.W                                   # a full window: every tick graduates
        sh._refresh_horizons()
        sh.enable_anomaly_list(cap=max(1024, 4 * capacity))
        return sh

    def _grow(self, capacity: int) -> None:
        old = self.shard
        new = self._new_shard(capacity)
        if old is not None:
            n = old.spec.n_series
            new.hist._store[:n].copy_(old.hist._store)
            new.hist.state.head, new.hist.state.length = old.hist.head, old.hist.length
            new.cur.data[:n].copy_(old.cur.data)
            new.cur.ticks = old.cur.ticks
            for name in ("threshold", "bound", "min_lower", "app_id"):
                getattr(new, name)[:n].copy_(getattr(old, name))
            new._refresh_horizons()
        self.keys.extend([None] * (capacity - len(self.keys)))
        self.shard = new

    def _clear_rows(self, rows: List[int]) -> None:
        if not rows:
            return
        idx = torch.tensor(rows, dtype=torch.long, device=self.device)
        self.shard.hist._store.index_fill_(0, idx, float("nan"))
        self.shard.cur.data.index_fill_(0, idx, float("nan"))

    def _assign_rows(self) -> List[Tuple[Key, int]]:
        """Free the rows of dead series, give pending series rows; returns the
        (key, row) pairs whose history must be loaded."""
        live = self.live_keys()
        dead = [k for k in self.rows if k not in live]
        freed = [self.rows.pop(k) for k in dead]
        for row in freed:
            self.keys[row] = None
        self.pending &= live
        new = sorted(k for k in self.pending if k not in self.rows)
        need = len(self.rows) + len(new)
        if self.shard is None or need > self.shard.spec.n_series:
            cap = max(self.min_capacity, self.shard.spec.n_series if self.shard is not None else 1)
            while cap < need:
                cap *= 2
            self._grow(cap)
        if freed:
            self._clear_rows(freed)
        free = [i for i, k in enumerate(self.keys) if k is None]
        out = []
        for key, row in zip(new, free):
            self.keys[row] = key
            self.rows[key] = row
            out.append((key, row))
        if dead or new:
            self._table = None
            self._refresh_apps()
        return out

    def _refresh_apps(self) -> None:
        """App roster of the live series (index = row of the per-app counters)."""
        names = sorted({(k[2], k[3]) for k in self.rows})
        if list(self.apps) != names:
            self.apps = {a: i for i, a in enumerate(names)}
            self.roster_version += 1
            self.roster_log.mark_reset()  # renumbered: consumers re-read the table
        sh = self.shard
        if sh.app_stats.shape[0] < max(1, len(self.apps)):
            cap = sh.app_stats.shape[0]
            while cap < len(self.apps):
                cap *= 2
            sh.app_stats = torch.zeros((cap, 2), dtype=torch.int32, device=self.device)
        ids = np.zeros(sh.spec.n_series, dtype=np.int32)
        for k, row in self.rows.items():
            ids[row] = self.apps[(k[2], k[3])]
        sh.app_id.copy_(torch.from_numpy(ids))

    def _set_thresholds(self, assigned: List[Tuple[Key, int]]) -> None:
        aliases: Dict[Key, str] = {}
        for j in self.jobs.values():
            for a, k in j.series.items():
                aliases.setdefault(k, a)
        rows = torch.tensor([row for _, row in assigned], dtype=torch.long, device=self.device)
        th = [self.cfg.for_metric(aliases.get(k, ""), k[1]) for k, _ in assigned]
        sh = self.shard
        sh.threshold[rows] = torch.tensor([t.threshold for t in th], dtype=torch.float32, device=self.device)
        sh.bound[rows] = torch.tensor([t.bound for t in th], dtype=torch.int8, device=self.device)
        sh.min_lower[rows] = torch.tensor([t.min_lower_bound for t in th], dtype=torch.float32, device=self.device)
        sh.refresh_thresholds()

    def _key_tables(self) -> Dict[Tuple[str, str], native.KeyTable]:
        """Per metric family (endpoint, metric): (namespace, app) → row."""
        if self._table is None:
            fams: Dict[Tuple[str, str], List] = {}
            for k, row in self.rows.items():
                fams.setdefault((k[0], k[1]), []).append(((k[2], k[3]), row))
            self._table = {fam: native.KeyTable(v) for fam, v in fams.items()}
        return self._table

    def _staging(self, rows: int, cols: int) -> Tuple[torch.Tensor, np.ndarray]:
        """NaN-filled host staging block (pinned for the GPU: one async H2D)."""
        t = torch.full((rows, cols), float("nan"), dtype=torch.float32)
        if self.device.type == "cuda":
            t = t.pin_memory()
        return t, t.numpy()

    # ------------------------------------------------------------------ data
    async def _fetch_into(self, reqs: List[Tuple[str, float, int, int]], out: np.ndarray,
                          tables: Dict[Tuple[str, str], native.KeyTable], fams: List[Tuple[str, str]]) -> List[bool]:
        """``reqs``: (url, start, n_points, col0) per query, ``fams`` the family of
        each; every response is decoded by the keyed native scatter into ``out``.
        Returns per request whether it was fetched and decoded."""
        return await fetch_decode(self.prom, reqs, [tables[f] for f in fams], out, self.step, self.decode_threads)

    async def _load_history(self, assigned: List[Tuple[Key, int]]) -> Set[Key]:
        """Fetch R + W points ending at ``t_last`` for the given series only, in
        (time chunk x app group) queries, into a pinned block; one H2D.  Returns
        the keys whose load had a failed query (they stay pending: retried next
        tick instead of keeping a NaN week)."""
        if not assigned:
            return set()
        n_pts = self.R + self.W
        first = self.t_last - (n_pts - 1) * self.step
        by_fam: Dict[Tuple[str, str], List[Tuple[Key, int]]] = {}
        for i, (key, _row) in enumerate(assigned):
            by_fam.setdefault((key[0], key[1]), []).append((key, i))
        block_t, block = self._staging(len(assigned), n_pts)
        reqs, fams, tables, groups = [], [], {}, []
        for fam, items in by_fam.items():
            tables[fam] = native.KeyTable([((k[2], k[3]), i) for k, i in items])
            for g in range(0, len(items), self.apps_per_query):
                grp = items[g:g + self.apps_per_query]
                sel = (f'{fam[1]}{{namespace=~"{_re_alt({k[2] for k, _ in grp})}",'
                       f'app=~"{_re_alt({k[3] for k, _ in grp})}"}}')
                for c0 in range(0, n_pts, self.chunk_pts):
                    n = min(self.chunk_pts, n_pts - c0)
                    s = first + c0 * self.step
                    url = (f"{fam[0]}query_range?query={quote(sel, safe='')}&start={int(s)}"
                           f"&end={int(s + (n - 1) * self.step)}&step={int(self.step)}")
                    reqs.append((url, s, n, c0))
                    fams.append(fam)
                    groups.append([k for k, _ in grp])
        self.history_queries += len(reqs)
        ok = await self._fetch_into(reqs, block, tables, fams)
        self.shard.load_rows(torch.tensor([row for _, row in assigned], dtype=torch.long),
                             block_t.to(self.device, non_blocking=True))
        self._set_thresholds(assigned)
        return {k for good, keys in zip(ok, groups) if not good for k in keys}

    async def _apply_changes(self) -> None:
        assigned = self._assign_rows()
        if self.shard is not None and self.t_last == 0.0:
            self.t_last = float(np.floor(self.clock() / self.step) * self.step)
        # rows whose history load failed earlier are still pending: load them again
        assigned = assigned + [(k, self.rows[k]) for k in sorted(self.pending)
                               if k in self.rows and k not in {a for a, _ in assigned}]
        if assigned:
            failed = await self._load_history(assigned)
            self.pending -= {k for k, _ in assigned if k not in failed}

    async def _ingest_new(self, now: float) -> None:
        t_new = float(np.floor(now / self.step) * self.step)
        n_new = int(round((t_new - self.t_last) / self.step))
        if n_new <= 0 or not self.rows:
            return
        if n_new > self.R:  # down for more than the whole history: reload every row
            self.t_last = t_new
            assigned = sorted(self.rows.items(), key=lambda kv: kv[1])
            failed = await self._load_history(assigned)
            self.pending |= failed
            return
        tables = self._key_tables()
        block_t, block = self._staging(self.shard.spec.n_series, n_new)
        s = self.t_last + self.step
        reqs, fams = [], []
        for fam in tables:
            for c0 in range(0, n_new, self.chunk_pts):  # catch-up after an outage: time chunks
                n = min(self.chunk_pts, n_new - c0)
                st = s + c0 * self.step
                url = (f"{fam[0]}query_range?query={quote(fam[1], safe='')}&start={int(st)}"
                       f"&end={int(st + (n - 1) * self.step)}&step={int(self.step)}")
                reqs.append((url, st, n, c0))
                fams.append(fam)
        ok = await self._fetch_into(reqs, block, tables, fams)
        if not all(ok):
            log.warning("%d of %d tick queries failed: the ring stays at %d, the next tick refetches",
                        ok.count(False), len(ok), int(self.t_last))
            return
        dev_block = block_t.to(self.device, non_blocking=True)
        for k in range(n_new):
            self.shard.ingest_tick(dev_block[:, k:k + 1].contiguous())
        self.t_last = t_new

    # ------------------------------------------------------------------ tick
    async def tick(self) -> Dict[str, str]:
        """One scoring tick over every continuous series; returns job → status written."""
        await self._apply_changes()
        written: Dict[str, str] = {}
        if self.shard is None or not self.rows:
            if self.shard is not None:
                self.shard.app_stats.zero_()
            return written
        t0 = time.perf_counter()
        now = self.clock()
        await self._ingest_new(now)
        out = self.shard.score()
        C = self.W
        col = (self.shard.cur.ticks - 1) % C
        verdict = out["verdict"].cpu().numpy()
        upper = out["upper"][:, col].float().cpu().numpy() if "upper" in out else None
        lower = out["lower"][:, col].float().cpu().numpy() if "lower" in out else None
        points: Dict[int, List[Tuple[float, float]]] = {}
        ab = self.shard.anomalies
        overflow = False
        if ab is not None:  # K9 device-side compaction: only the anomalies come back
            rows, cols, vals, overflow = ab.fetch()
        if ab is None or overflow:
            x = self.shard.cur.data.float().cpu().numpy()
            up = out["upper"].float().cpu().numpy()
            lo = out["lower"].float().cpu().numpy()
            b = self.shard.bound.cpu().numpy().astype(np.int64)[:, None]
            flag = (((b & 1) != 0) & (x > up)) | (((b & 2) != 0) & (x < lo))
            flag &= (verdict == 1)[:, None]
            rows, cols = np.nonzero(flag)
            vals = x[rows, cols]
        for rr, cc, vv in zip(rows.tolist(), cols.tolist(), vals.tolist()):
            age = (col - cc) % C
            points.setdefault(rr, []).append((self.t_last - age * self.step, vv))
        self.ticks += 1
        self.metrics.tick.observe(time.perf_counter() - t0)
        self.metrics.series_scored.inc(len(self.rows))
        for jid, job in list(self.jobs.items()):
            anomaly = {}
            for alias, key in job.series.items():
                row = self.rows.get(key)
                if row is None:
                    continue
                ep, metric, ns, app = key
                if upper is not None and ns:
                    self.metrics.export_band(metric, ns, app, float(upper[row]), float(lower[row]),
                                             self.t_last if verdict[row] == 1 else None)
                if verdict[row] == 1:
                    flat: List[float] = []
                    for ts, v in sorted(points.get(row, [])):
                        flat += [ts, float(v)]
                    anomaly[alias] = {"tags": "", "values": flat}
            if anomaly:
                status, reason = r.ST_COMPLETED_UNHEALTH, "anomaly detected in " + ",".join(sorted(anomaly))
            elif now >= job.end_ts:
                status, reason = r.ST_COMPLETED_HEALTH, ""
            else:
                status, reason = r.ST_PREPROCESS_INPROGRESS, ""
            fields = {"status": status, "reason": reason, "modified_ts": now,
                      "processingContent": f"streamed by {self.worker_id}"}
            if anomaly:
                fields["anomalyInfo"] = json.dumps(anomaly)
            if status in r.TERMINAL_STATUSES:
                fields["claimed_by"] = ""
            ok = self.store.update(jid, fields, expect_claimed_by=self.worker_id)
            if not ok or status in r.TERMINAL_STATUSES:
                del self.jobs[jid]  # finished, or another worker took the lease
                if ok:
                    self.metrics.jobs.labels(status=status).inc()
            written[jid] = status
        return written

    def app_table(self) -> Tuple[List[Tuple[str, str]], torch.Tensor]:
        """(app roster, ``[A, 2]`` int32 device counters of the last tick:
        anomalous series, scored series)."""
        return list(self.apps), self.app_counts()

    def roster_names(self) -> List[Tuple[str, str]]:
        return list(self.apps)

    def app_counts(self) -> torch.Tensor:
        if self.shard is None:
            return torch.zeros((len(self.apps), 2), dtype=torch.int32, device=self.device)
        return self.shard.app_stats[:len(self.apps)]

    # ------------------------------------------------------------------ checkpoint / resume
    def save_snapshot(self, path: str) -> bool:
        """Checkpoint the resident shard (history ring, windows, last fit) with
        the series key of every row (``brain/checkpoint.py``)."""
        if self.shard is None or self.pending:
            return False
        from . import checkpoint as ck
        ck.save_streaming_shard(self.shard, path, extra={"keys": [list(k) if k else None for k in self.keys],
                                                         "t_last": float(self.t_last), "step": self.step})
        return True

    def restore_snapshot(self, path: str) -> bool:
        """Adopt a snapshot instead of re-fetching a week of history per series:
        only when it holds every series of the leased jobs, with the same
        geometry, and is younger than half the ring (the next tick then catches
        up the missed points); otherwise rows are loaded from Prometheus."""
        import os
        if not path or not os.path.exists(path):
            return False
        from . import checkpoint as ck
        try:
            shard = ck.load_streaming_shard(path, self.cfg, self.device)
        except (ValueError, KeyError, OSError) as e:
            log.warning("ignoring snapshot %s: %s", path, e)
            return False
        ex = shard.checkpoint_extra
        keys = [tuple(k) if k else None for k in ex.get("keys", [])]
        snap_rows = {k: i for i, k in enumerate(keys) if k is not None}
        if (set(snap_rows) != self.live_keys() or ex.get("step") != self.step or shard.spec.ring_len != self.R
                or shard.spec.window != self.W or self.clock() - float(ex.get("t_last", 0)) > self.R * self.step / 2):
            return False
        shard.enable_anomaly_list(cap=max(1024, 4 * len(keys)))
        self.shard, self.t_last = shard, float(ex["t_last"])
        self.keys, self.rows, self.pending = keys, snap_rows, set()
        self._table = None
        self._refresh_apps()
        return True

    async def run_forever(self, stop: Optional[asyncio.Event] = None, period: Optional[float] = None,
                          snapshot: Optional[str] = None, snapshot_every: int = 60) -> None:
        """Tick every ``period`` seconds; with ``snapshot``, resume from it on the
        first tick and re-save it every ``snapshot_every`` ticks and at exit."""
        period = self.step if period is None else period
        first = True
        while stop is None or not stop.is_set():
            try:
                self.sync()
                if first and snapshot and self.restore_snapshot(snapshot):
                    log.info("resumed %d series from snapshot %s", len(self.rows), snapshot)
                first = False
                await self.tick()
                if snapshot and snapshot_every > 0 and self.ticks % snapshot_every == 0:
                    self.save_snapshot(snapshot)
            except Exception as e:  # noqa: BLE001 - keep monitoring
                log.exception("streaming tick failed: %s", e)
            try:
                await asyncio.wait_for(stop.wait(), timeout=period) if stop else await asyncio.sleep(period)
            except asyncio.TimeoutError:
                pass
        if snapshot:
            self.save_snapshot(snapshot)
