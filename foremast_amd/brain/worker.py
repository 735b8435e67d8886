"""The brain job loop (foremast-brain, absent from the reference repo).

Reconstructed from ``docs/guides/design.md:33-43`` and the request state
diagram::

    claim   : status in {initial, reprogress}, or in progress longer than
              MAX_STUCK_IN_SECONDS (takeover)   → preprocess_inprogress
    fetch   : historical / baseline / current range vectors (concurrent)
    score   : one batched GPU pass over every (job, metric) of the cycle
    verdict : anomaly                  → completed_unhealth   (fail fast)
              endTime reached, healthy → completed_health
              no current data at end   → completed_unknown
              otherwise                → reprogress (re-claimed next cycle)
    export  : foremastbrain:<metric>_{upper,lower,anomaly} gauges

Writes go through the job store with ``expect_claimed_by`` so a worker that
lost its lease (stuck-job takeover by another brain) cannot overwrite the
new owner's result.
"""

from __future__ import annotations

import asyncio
import json
import logging
import os
import socket
import time
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Tuple

import numpy as np

from ..api import rest as r
from ..promql.client import FetchError, PromClient, Series
from ..promql.selector import SelectorError, parse_selector
from ..service import urls
from ..store import JobStore
from ..utils.config import BrainConfig
from ..utils.metrics import BrainMetrics
from ..utils.timeutil import TimeFormatError, parse_rfc3339
from .batch import BatchScorer, MetricTask, TaskResult

# recorded split families (deploy/rules.py SPLIT_PREFIXES): selector prefix -> split label
SPLIT_PREFIXES = {"namespace_pod_caller:": "caller", "namespace_app_caller:": "caller",
                  "namespace_app_caller_per_pod:": "caller", "namespace_pod_uri:": "uri",
                  "namespace_app_uri:": "uri", "namespace_app_uri_per_pod:": "uri"}


def split_label_of(metric: str) -> str:
    for pfx, label in SPLIT_PREFIXES.items():
        if metric.startswith(pfx):
            return label
    return ""

log = logging.getLogger("foremast.brain")


@dataclass
class JobPlan:
    doc: Dict[str, Any]
    end_ts: float
    current: Dict[str, str] = field(default_factory=dict)
    baseline: Dict[str, str] = field(default_factory=dict)
    historical: Dict[str, str] = field(default_factory=dict)
    sources: Dict[str, str] = field(default_factory=dict)
    error: str = ""


def _selector_info(url: str) -> Tuple[str, str, str]:
    try:
        q = urls.parse_prometheus_url(url)["query"]
        sel = parse_selector(str(q))
    except (urls.ConfigError, SelectorError):
        return "", "", ""
    labels = {k: v for k, op, v in sel.matchers if op == "="}
    return sel.name, labels.get("namespace", ""), labels.get("app", "")


def _grid(url: str) -> Tuple[float, float, float]:
    p = urls.parse_prometheus_url(url)
    return float(p["start"]), float(p["end"]), float(p["step"])


class BrainWorker:
    def __init__(self, store: JobStore, cfg: Optional[BrainConfig] = None, prom: Optional[PromClient] = None,
                 scorer: Optional[BatchScorer] = None, worker_id: Optional[str] = None,
                 clock=time.time, metrics: Optional[BrainMetrics] = None, batch_limit: int = 256,
                 exclude_strategies: Tuple[str, ...] = ()) -> None:
        self.store = store
        self.cfg = cfg or BrainConfig.from_env()
        self.prom = prom or PromClient()
        self.scorer = scorer or BatchScorer(self.cfg)
        self.worker_id = worker_id or f"{socket.gethostname()}-{os.getpid()}"
        self.clock = clock
        self.metrics = metrics or BrainMetrics()
        self.batch_limit = batch_limit
        # strategies another component owns (the streaming monitor takes "continuous")
        self.exclude = {x.lower() for x in exclude_strategies}
        self.lstm = None  # LstmJobScorer, created on first multivariate LSTM job
        self.downstream = None  # per-caller joint LstmJobScorer (fp8), created on first downstream job

    def _claimable(self, d: Dict[str, Any]) -> bool:
        """Strategies a resident engine owns are skipped — except the jobs that
        engine cannot key: continuous jobs with per-caller series
        (streaming.is_streamable) and rollout jobs outside the rollout table
        (rollout.is_rollout_keyable: other data sources, split families,
        multi-metric algorithms)."""
        s = (d.get("strategy") or "").lower()
        if s not in self.exclude:
            return True
        if s == "continuous":
            from .streaming import is_streamable
            return not is_streamable(d)
        from .rollout import STRATEGIES, is_rollout_keyable
        return s in STRATEGIES and not is_rollout_keyable(d, self.cfg)

    # ------------------------------------------------------------------ planning
    def plan(self, doc: Dict[str, Any]) -> JobPlan:
        try:
            end_ts = parse_rfc3339(doc.get("endTime", "")).timestamp()
        except TimeFormatError:
            end_ts = 0.0
        p = JobPlan(doc=doc, end_ts=end_ts)
        try:
            p.current = urls.parse_config(doc.get("currentConfig", ""))
            p.baseline = urls.parse_config(doc.get("baselineConfig", ""))
            p.historical = urls.parse_config(doc.get("historicalConfig", ""))
            p.sources = urls.parse_config(doc.get("currentMetricStore", ""))
        except urls.ConfigError as e:
            p.error = f"bad config: {e}"
        if not p.current and not p.error:
            p.error = "no current metric config"
        unsupported = [a for a, s in p.sources.items() if s and s != r.DATASOURCE_PROMETHEUS]
        if unsupported and not p.error:
            p.error = "unsupported data source for " + ",".join(sorted(unsupported))
        return p

    # ------------------------------------------------------------------ one cycle
    async def cycle(self) -> int:
        t0 = time.perf_counter()
        now = self.clock()
        only = self._claimable if self.exclude else None
        docs = self.store.claim(self.worker_id, now=now, max_stuck_s=self.cfg.max_stuck_seconds,
                                limit=self.batch_limit, only=only)
        if not docs:
            return 0
        plans = [self.plan(d) for d in docs]
        # fetch everything concurrently
        reqs: List[Tuple[int, str, str, str]] = []  # (plan, category, alias, url)
        for i, p in enumerate(plans):
            if p.error:
                continue
            for cat, m in (("current", p.current), ("baseline", p.baseline), ("historical", p.historical)):
                for alias, url in m.items():
                    reqs.append((i, cat, alias, url))
        fetched = await self.prom.fetch_many([u for _, _, _, u in reqs])
        data: Dict[Tuple[int, str, str], Any] = {}
        for (i, cat, alias, _), res in zip(reqs, fetched):
            data[(i, cat, alias)] = res
        tasks: List[MetricTask] = []
        owners: List[int] = []
        fetch_errors: Dict[int, List[str]] = {}
        for i, p in enumerate(plans):
            if p.error:
                continue
            for alias in sorted(p.current):
                for task in self._build_tasks(i, p, alias, data, fetch_errors):
                    tasks.append(task)
                    owners.append(i)
        results: List[TaskResult] = self.scorer.score(tasks) if tasks else []
        per_job: Dict[int, List[Tuple[MetricTask, TaskResult]]] = {}
        for t, res, i in zip(tasks, results, owners):
            per_job.setdefault(i, []).append((t, res))
        self._multivariate(plans, per_job)
        for i, p in enumerate(plans):
            self._finish(p, per_job.get(i, []), fetch_errors.get(i, []), now)
        self.metrics.detect_latency.observe(time.perf_counter() - t0)
        self.metrics.series_scored.inc(len(tasks))
        return len(docs)

    def _build_tasks(self, i: int, p: JobPlan, alias: str, data, errors) -> List[MetricTask]:
        """One task per metric alias — or, for a split alias (``metricType:
        downstream`` / ``api``), one per calling service / request path found in
        the history or the current window."""
        cur = data.get((i, "current", alias))
        hist = data.get((i, "historical", alias))
        base = data.get((i, "baseline", alias))
        if isinstance(cur, Exception):
            errors.setdefault(i, []).append(f"{alias}: current fetch failed")
            cur = []
        if isinstance(hist, Exception) or hist is None:
            errors.setdefault(i, []).append(f"{alias}: historical fetch failed")
            return []
        if base is not None and isinstance(base, Exception):
            base = None
        hurl = p.historical.get(alias, "")
        metric, ns, app = _selector_info(hurl)
        label = split_label_of(metric)
        if not label:
            return [self._task(p, alias, metric, ns, app, hurl, hist, cur or [], base)]
        groups = sorted({s.labels.get(label, "") for s in list(hist) + list(cur or [])})

        def of(series, c):
            return [s for s in series if s.labels.get(label, "") == c]
        out = []
        for c in groups:
            t = self._task(p, f"{alias}[{label}={c}]", metric, ns, app, hurl, of(hist, c), of(cur or [], c),
                           of(base, c) if base is not None else None)
            t.caller, t.base_alias, t.split_label = c, alias, label
            out.append(t)
        return out

    def _task(self, p: JobPlan, alias: str, metric: str, ns: str, app: str, hurl: str, hist, cur,
              base) -> MetricTask:
        start, end, step = _grid(hurl)
        T = int(round((end - start) / step)) + 1
        sums = np.zeros(T)
        cnt = np.zeros(T)
        for s in hist:  # several series (e.g. per pod) → mean per timestamp
            idx = np.rint((s.ts - start) / step).astype(np.int64)
            ok = (idx >= 0) & (idx < T) & ~np.isnan(s.values)
            np.add.at(cnt, idx[ok], 1)
            np.add.at(sums, idx[ok], s.values[ok].astype(np.float64))
        h = np.where(cnt > 0, sums / np.maximum(cnt, 1), np.nan).astype(np.float32)
        cts, cvs, tags = [], [], []
        for s in cur:
            cts.append(s.ts)
            cvs.append(s.values)
            tags += [s.labels.get("pod", s.labels.get("app", ""))] * len(s.ts)
        cur_ts = np.concatenate(cts) if cts else np.zeros(0)
        cur_vals = np.concatenate(cvs).astype(np.float32) if cvs else np.zeros(0, dtype=np.float32)
        base_vals = None
        if base:
            base_vals = np.concatenate([s.values for s in base]).astype(np.float32)
        th = self.cfg.for_metric(alias, metric)
        return MetricTask(job_id=p.doc["id"], alias=alias, metric=metric or alias, namespace=ns, app=app,
                          step=step, hist=h, hist_end=start + (T - 1) * step, cur_ts=cur_ts, cur_vals=cur_vals,
                          cur_tags=tags, base_vals=base_vals, threshold=th.threshold, bound=th.bound,
                          min_lower=th.min_lower_bound, base_alias=alias)

    def _multivariate(self, plans: List[JobPlan], per_job) -> None:
        """Joint models on top of the per-metric verdicts: ``bivariate_normal``
        (>= 2 metrics, first two aliases), ``lstm`` (>= 2 metrics), or
        ``auto`` = the design doc's dispatch (2 metrics → bivariate normal,
        3+ → LSTM autoencoder; ``docs/guides/design.md:76-84``)."""
        self._downstream(per_job)
        algo = self.cfg.algorithm
        if algo not in ("bivariate_normal", "lstm", "auto"):
            return
        # per-caller (downstream) tasks are scored jointly per caller by _downstream
        per_job = {i: [(t, r_) for t, r_ in items if not t.split_label] for i, items in per_job.items()}
        lstm_jobs = [i for i, items in per_job.items()
                     if (algo == "lstm" and len(items) >= 2) or (algo == "auto" and len(items) >= 3)]
        if lstm_jobs:
            self._score_lstm(per_job, lstm_jobs)
        if algo == "lstm":
            return
        pairs, owners = [], []
        for i, items in per_job.items():
            if len(items) == 2 or (algo == "bivariate_normal" and len(items) >= 2):
                (ta, _), (tb, _) = items[0], items[1]
                pairs.append((ta, tb))
                owners.append(i)
        for i, (verdict, pts) in zip(owners, self.scorer.score_bivariate(pairs)):
            ta, ra = per_job[i][0]
            tb, rb = per_job[i][1]
            if verdict == 1:
                ra.verdict = max(ra.verdict, 1)
                ra.anomalies = [(ts, v, "") for ts, v in pts]
                ra.model = rb.model = "bivariate_normal"

    def _downstream(self, per_job) -> None:
        """Downstream impact / API level: for every caller (or request path) of the
        deployed app with >= 2 monitored metrics (e.g. latency + error rate), its metrics are
        scored JOINTLY by an LSTM autoencoder (fp8 e4m3 MFMA scoring on the GPU),
        keyed per (namespace, app, caller) in the model cache; a joint anomaly
        marks each of the caller's metrics anomalous at the flagged timestamps.
        ``ML_DOWNSTREAM_ALGORITHM=none`` keeps only the per-metric verdicts."""
        if self.cfg.downstream_algorithm == "none":
            return
        from .multivariate import LstmJobScorer, ModelCache, align_job
        for i, items in per_job.items():
            by_caller: Dict[Tuple[str, str], List[Tuple[MetricTask, TaskResult]]] = {}
            for t, res in items:
                if t.split_label:
                    by_caller.setdefault((t.split_label, t.caller), []).append((t, res))
            for (label, caller), group in sorted(by_caller.items()):
                group = sorted(group, key=lambda tr: tr[0].base_alias)
                if len(group) < 2:
                    continue
                tasks = [t for t, _ in group]
                hist, cts, cur = align_job(tasks)
                if not len(cts):
                    continue
                if self.downstream is None:
                    self.downstream = LstmJobScorer(device=self.scorer.device,
                                                    cache=ModelCache(self.cfg.max_cache_size),
                                                    threshold=self.cfg.lstm_threshold, fp8=True)
                key = self.downstream.cache.key(tasks[0].namespace, f"{tasks[0].app}@{label}={caller}",
                                                [t.base_alias for t in tasks])
                verdict, bad, _z = self.downstream.score_job(key, hist, cts, cur, now=self.clock())
                for f, (t, res) in enumerate(group):
                    if verdict == 1:
                        res.verdict = 1
                        seen = {(ts, tag) for ts, _, tag in res.anomalies}
                        res.anomalies = res.anomalies + [(float(cts[j]), float(cur[j, f]), "joint")
                                                         for j in bad if (float(cts[j]), "joint") not in seen]
                        res.model = (res.model + "+lstm_fp8") if "lstm" not in res.model else res.model

    def _score_lstm(self, per_job, jobs: List[int]) -> None:
        from .multivariate import LstmJobScorer, ModelCache, align_job
        if self.lstm is None:
            self.lstm = LstmJobScorer(device=self.scorer.device, cache=ModelCache(self.cfg.max_cache_size),
                                      threshold=self.cfg.lstm_threshold)
        for i in jobs:
            items = sorted(per_job[i], key=lambda tr: tr[0].alias)
            tasks = [t for t, _ in items]
            hist, cts, cur = align_job(tasks)
            key = self.lstm.cache.key(tasks[0].namespace, tasks[0].app, [t.alias for t in tasks])
            verdict, bad, _z = self.lstm.score_job(key, hist, cts, cur, now=self.clock())
            for f, (t, res) in enumerate(items):
                res.model = "lstm"
                if verdict == 1:
                    res.verdict = 1
                    res.anomalies = [(float(cts[j]), float(cur[j, f]), "") for j in bad]

    def _finish(self, p: JobPlan, items: List[Tuple[MetricTask, TaskResult]], errors: List[str], now: float):
        doc_id = p.doc["id"]
        if p.error:
            self._write(doc_id, r.ST_PREPROCESS_FAILED, p.error)
            return
        anomaly: Dict[str, Dict[str, Any]] = {}
        any_current = False
        for t, res in items:
            any_current |= bool(len(t.cur_vals))
            if len(res.upper) and t.namespace:
                last_anom = res.anomalies[-1][0] if res.anomalies else None
                self.metrics.export_band(t.metric, t.namespace, t.app, float(res.upper[-1]),
                                         float(res.lower[-1]), last_anom)
            if res.verdict == 1 and res.anomalies:
                vals: List[float] = []
                for ts, v, _ in sorted(res.anomalies):
                    vals += [ts, v]
                tags = sorted({tag for _, _, tag in res.anomalies if tag})
                if t.split_label:  # downstream / API level: name the caller or the request path
                    tags = [f"{t.split_label}={t.caller}"] + [x for x in tags if x != "joint"]
                tags = ",".join(tags)
                anomaly[t.alias] = {"tags": tags, "values": vals}
        if anomaly:
            self._write(doc_id, r.ST_COMPLETED_UNHEALTH,
                        "anomaly detected in " + ",".join(sorted(anomaly)), anomaly)
            return
        if now >= p.end_ts:
            if any_current and not errors:
                self._write(doc_id, r.ST_COMPLETED_HEALTH, "")
            else:
                reason = "; ".join(errors) or "no current metric data"
                self._write(doc_id, r.ST_COMPLETED_UNKNOWN, reason)
            return
        self._write(doc_id, r.ST_REPROGRESS, "; ".join(errors),
                    not_before=now + self.cfg.poll_seconds)

    def _write(self, doc_id: str, status: str, reason: str, anomaly: Optional[Dict] = None,
               not_before: float = 0.0) -> None:
        fields: Dict[str, Any] = {"status": status, "reason": reason, "not_before": not_before,
                                  "processingContent": f"scored by {self.worker_id}"}
        if anomaly:
            fields["anomalyInfo"] = json.dumps(anomaly)
        if status in r.TERMINAL_STATUSES:
            fields["claimed_by"] = ""
        ok = self.store.update(doc_id, fields, expect_claimed_by=self.worker_id)
        if ok and status in r.TERMINAL_STATUSES:
            self.metrics.jobs.labels(status=status).inc()

    async def run_forever(self, stop: Optional[asyncio.Event] = None) -> None:
        while stop is None or not stop.is_set():
            try:
                n = await self.cycle()
            except Exception as e:  # noqa: BLE001 - keep the loop alive
                log.exception("brain cycle failed: %s", e)
                n = 0
            if n == 0:
                await asyncio.sleep(min(self.cfg.poll_seconds, 1.0))
