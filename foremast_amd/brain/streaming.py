"""Continuous monitoring on the streaming GPU engine.

Continuous jobs (``strategy: continuous`` — barrelman's ``monitorContinuously``,
``Barrelman.go:176-203``) ask the same question every minute for as long as
the job runs.  Instead of refetching and refitting each job independently
(what :class:`~foremast_amd.brain.worker.BrainWorker` does for one-shot
canary/rollout jobs), the :class:`StreamingMonitor` keeps every continuous
series resident in one :class:`~foremast_amd.brain.engine.StreamingShard`:

* history: 7 days at the query step in the HBM bf16 ring, loaded once per
  membership change with ONE range query per metric family (the bare
  recorded series name returns every app's series; the response is parsed by
  the native C++ matrix parser and scattered by ``(namespace, app)``);
* every tick: one short range query per metric family for the newest point
  of all series → tick ingest kernel → one fused scoring launch for all
  series → per-job verdicts;
* jobs: leased from the job store with a strategy filter (the one-shot
  worker skips them), lease renewed each tick; any anomalous series finishes
  its job ``completed_unhealth`` with the anomalous point; past ``endTime``
  a job finishes ``completed_health``; band gauges are exported for the UI.
"""

from __future__ import annotations

import asyncio
import json
import logging
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple
from urllib.parse import quote

import numpy as np
import torch

from ..api import rest as r
from ..promql.client import PromClient
from ..promql.selector import SelectorError, parse_selector
from ..service import urls
from ..store.jobstore import JobStore
from ..utils.config import BrainConfig
from ..utils.metrics import BrainMetrics
from ..utils.timeutil import TimeFormatError, parse_rfc3339
from .engine import ShardSpec, StreamingShard

log = logging.getLogger("foremast.streaming")

STRATEGY_CONTINUOUS = "continuous"


def is_continuous(doc) -> bool:
    return (doc.get("strategy") or "").lower() == STRATEGY_CONTINUOUS


@dataclass
class StreamJob:
    doc: Dict
    end_ts: float
    series: Dict[str, int] = field(default_factory=dict)  # alias -> row


class StreamingMonitor:
    def __init__(self, store: JobStore, cfg: Optional[BrainConfig] = None, prom: Optional[PromClient] = None,
                 device=None, worker_id: str = "stream-0", metrics: Optional[BrainMetrics] = None,
                 ring_len: int = 10080, step: float = 60.0, window: int = 10, clock=time.time) -> None:
        self.store = store
        self.cfg = cfg or BrainConfig.from_env()
        self.prom = prom or PromClient()
        self.device = torch.device(device) if device is not None else (
            torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu"))
        self.worker_id = worker_id
        self.metrics = metrics or BrainMetrics()
        self.R, self.step, self.W = ring_len, step, window
        self.clock = clock
        self.jobs: Dict[str, StreamJob] = {}
        self.keys: List[Tuple[str, str, str, str]] = []  # (endpoint, metric, namespace, app)
        self.rows: Dict[Tuple[str, str, str, str], int] = {}
        self.shard: Optional[StreamingShard] = None
        self.dirty = False
        self.ticks = 0

    # ------------------------------------------------------------------ membership
    def _series_of(self, doc) -> Dict[str, Tuple[str, str, str, str]]:
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

    def sync(self) -> int:
        """Lease new continuous jobs; returns how many were added."""
        now = self.clock()
        docs = self.store.claim(self.worker_id, now=now, max_stuck_s=self.cfg.max_stuck_seconds, limit=10_000,
                                only=is_continuous)
        for d in docs:
            try:
                end_ts = parse_rfc3339(d.get("endTime", "")).timestamp()
            except TimeFormatError:
                end_ts = float("inf")
            job = StreamJob(doc=d, end_ts=end_ts)
            for alias, key in self._series_of(d).items():
                if key not in self.rows:
                    self.rows[key] = len(self.keys)
                    self.keys.append(key)
                    self.dirty = True
                job.series[alias] = self.rows[key]
            self.jobs[d["id"]] = job
        return len(docs)

    def _compact(self) -> None:
        """Drop series no job uses any more (after jobs finish)."""
        used = {row for j in self.jobs.values() for row in j.series.values()}
        if len(used) == len(self.keys):
            return
        keep = [k for k in self.keys if self.rows[k] in used]
        remap = {self.rows[k]: i for i, k in enumerate(keep)}
        self.keys = keep
        self.rows = {k: i for i, k in enumerate(keep)}
        for j in self.jobs.values():
            j.series = {a: remap[row] for a, row in j.series.items()}
        self.dirty = True

    # ------------------------------------------------------------------ data
    def _families(self) -> Dict[Tuple[str, str], List[int]]:
        fam: Dict[Tuple[str, str], List[int]] = {}
        for i, (ep, metric, _ns, _app) in enumerate(self.keys):
            fam.setdefault((ep, metric), []).append(i)
        return fam

    async def _fetch_grid(self, start: float, n: int) -> np.ndarray:
        """``[N, n]`` values on the grid ``start + k*step`` (NaN where missing):
        one range query per (endpoint, metric family)."""
        N = len(self.keys)
        out = np.full((N, n), np.nan, dtype=np.float32)
        fams = self._families()
        end = start + (n - 1) * self.step
        req = [f"{ep}query_range?query={quote(metric, safe='')}&start={int(start)}&end={int(end)}"
               f"&step={int(self.step)}" for (ep, metric) in fams]
        res = await self.prom.fetch_many(req)
        for (ep, metric), series in zip(fams, res):
            if isinstance(series, Exception):
                log.warning("fetch %s failed: %s", metric, series)
                continue
            for s in series:
                row = self.rows.get((ep, metric, s.labels.get("namespace", ""), s.labels.get("app", "")))
                if row is None:
                    continue
                idx = np.rint((s.ts - start) / self.step).astype(np.int64)
                ok = (idx >= 0) & (idx < n)
                out[row, idx[ok]] = s.values[ok]
        return out

    async def rebuild(self) -> None:
        """(Re)load every live series' history and prefill the current window."""
        self._compact()
        N = len(self.keys)
        self.dirty = False
        if N == 0:
            self.shard = None
            return
        now = self.clock()
        t_last = np.floor(now / self.step) * self.step
        first = t_last - (self.R + self.W - 1) * self.step
        grid = await self._fetch_grid(first, self.R + self.W)
        season = max(2, int(round(86400.0 / self.step)))
        algo = self.cfg.algorithm if self.cfg.algorithm in ("holt_winters", "exponential_smoothing",
                                                            "double_exponential_smoothing", "moving_average",
                                                            "moving_average_all") else "moving_average_all"
        if algo == "holt_winters" and self.R < 2 * season:
            algo = "double_exponential_smoothing"
        aliases = [""] * N
        for j in self.jobs.values():
            for a, row in j.series.items():
                aliases[row] = a
        th = [self.cfg.for_metric(aliases[i], self.keys[i][1]) for i in range(N)]
        dev = self.device
        spec = ShardSpec(n_series=N, ring_len=self.R, season=season, pods=1, window=self.W, algorithm=algo,
                         pairwise="NONE", dtype=torch.bfloat16 if dev.type == "cuda" else torch.float32)
        self.shard = StreamingShard(
            spec, self.cfg, dev,
            threshold=torch.tensor([t.threshold for t in th], dtype=torch.float32, device=dev),
            bound=torch.tensor([t.bound for t in th], dtype=torch.int8, device=dev),
            min_lower=torch.tensor([t.min_lower_bound for t in th], dtype=torch.float32, device=dev))
        self.shard.enable_anomaly_list(cap=max(1024, 4 * N))
        self.shard.load_history(torch.from_numpy(np.ascontiguousarray(grid[:, :self.R])))
        for k in range(self.W):
            self.shard.ingest_tick(torch.from_numpy(np.ascontiguousarray(grid[:, self.R + k:self.R + k + 1])).to(dev))
        self.t_last = t_last

    # ------------------------------------------------------------------ tick
    async def tick(self) -> Dict[str, str]:
        """One scoring tick over every continuous series; returns job → status written."""
        if self.dirty or self.shard is None:
            await self.rebuild()
        written: Dict[str, str] = {}
        if self.shard is None:
            return written
        t0 = time.perf_counter()
        now = self.clock()
        t_new = np.floor(now / self.step) * self.step
        n_new = int(round((t_new - self.t_last) / self.step))
        if n_new > 0:
            grid = await self._fetch_grid(self.t_last + self.step, min(n_new, self.W))
            for k in range(grid.shape[1]):
                self.shard.ingest_tick(torch.from_numpy(np.ascontiguousarray(grid[:, k:k + 1])).to(self.device))
            self.t_last = t_new
        out = self.shard.score()
        C = self.W
        col = (self.shard.cur.ticks - 1) % C
        verdict = out["verdict"].cpu().numpy()
        upper = out["upper"][:, col].float().cpu().numpy() if "upper" in out else None
        lower = out["lower"][:, col].float().cpu().numpy() if "lower" in out else None
        # anomalous points of the current window per series: (timestamp, value) pairs
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
        self.metrics.series_scored.inc(len(self.keys))
        for jid, job in list(self.jobs.items()):
            anomaly = {}
            for alias, row in job.series.items():
                ep, metric, ns, app = self.keys[row]
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
                self.dirty = True
                if ok:
                    self.metrics.jobs.labels(status=status).inc()
            written[jid] = status
        return written

    # ------------------------------------------------------------------ checkpoint / resume
    def save_snapshot(self, path: str) -> bool:
        """Checkpoint the resident shard (history ring, windows, last fit) with
        the series keys it serves (``brain/checkpoint.py``)."""
        if self.shard is None:
            return False
        from . import checkpoint as ck
        ck.save_streaming_shard(self.shard, path, extra={"keys": [list(k) for k in self.keys],
                                                         "t_last": float(self.t_last), "step": self.step})
        return True

    def restore_snapshot(self, path: str) -> bool:
        """Adopt a snapshot instead of re-fetching a week of history per series:
        only when it serves exactly the series of the leased jobs, with the same
        geometry, and is younger than half the ring (the next tick then catches
        up the missed points); otherwise the next tick rebuilds from Prometheus."""
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
        keys = [tuple(k) for k in ex.get("keys", [])]
        if (keys != self.keys or ex.get("step") != self.step or shard.spec.ring_len != self.R
                or shard.spec.window != self.W or self.clock() - float(ex.get("t_last", 0)) > self.R * self.step / 2):
            return False
        shard.enable_anomaly_list(cap=max(1024, 4 * len(keys)))
        self.shard, self.t_last, self.dirty = shard, float(ex["t_last"]), False
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
                    log.info("resumed %d series from snapshot %s", len(self.keys), snapshot)
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
