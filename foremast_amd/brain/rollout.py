"""One-shot canary / rollingUpdate jobs on the resident GPU engine.

The reference brain answers a rollout job by re-running the whole judgement
every cycle until ``endTime`` (``docs/guides/design.md:35,43``): fetch the
7-day history of each metric, the baseline pods' window (canary only) and the
new pods' window so far (``metricsquery.go:52-79``), fit the historical
model, run the pairwise test, lower the threshold if baseline and current
differ, detect.  :class:`RolloutMonitor` serves the same jobs from resident
state instead:

* admission (once per job, batched over every job claimed in a tick): the
  history comes from the node's resident ring (:mod:`.resident`; fetched only
  for series the node has never held), the model is fitted ONCE on the
  history ending at the job's start — the reference job's historical window is
  fixed at creation, so refitting it every cycle would recompute the same
  model — and reduced to a forecast state per (job, metric) row: level,
  trend, the 16 forecast offsets of the current window's horizons, sigma,
  fitted grid point (h-step variance) and valid points.  The baseline pods'
  window ``[start - W, start]`` is fetched once, batched by pod family;
* every tick: ONE range query per pod metric family for the newest minute of
  every pod of every running job → native keyed decode (``(namespace, pod)`` →
  row x pod) → one H2D → scatter kernel into each row's window at its own
  job-minute column → rank tests (MW-U / Wilcoxon / Kruskal, pods pooled) of
  baseline vs current → band / verdict / per-app counters / compacted anomaly
  list from the cached state (one launch, ``hw_detect_params_kernel``) → D2H;
* verdicts follow the reference state machine: an anomalous metric finishes
  the job ``completed_unhealth`` with its points and pod tags (fail fast);
  past ``endTime`` it finishes ``completed_health`` (current data seen) or
  ``completed_unknown``; in between the job stays leased — the engine renews
  all of its leases with one store heartbeat per tick instead of a write per
  job — and nothing is written;
* rows are freed when their job finishes; band gauges are read from the last
  tick's host arrays at scrape time.

Jobs the resident engine cannot key (non-Prometheus sources, per-caller /
per-uri families, selectors that are not plain pod lists, multi-metric
algorithms) stay with :class:`~foremast_amd.brain.worker.BrainWorker`
(:func:`is_rollout_keyable`).
"""

from __future__ import annotations

import heapq
import json
import logging
import math
import re
import time
from collections import OrderedDict
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Set, Tuple
from urllib.parse import unquote

import numpy as np
import torch

from ..api import rest as r
from ..ingest import native
from ..models import decompose as dec_ref
from ..models import detect as det_ref
from ..models import moving_average as ma_ref
from ..models import pairwise as pw_ref
from ..models import smoothing as sm_ref
from ..promql.selector import SelectorError, parse_selector
from ..service import urls
from ..store.jobstore import JobStore
from ..utils.config import BrainConfig
from ..utils.metrics import BrainMetrics
from ..utils.timeutil import TimeFormatError, parse_rfc3339
from .resident import Key, ResidentHistory, fetch_decode, range_url, re_alt

log = logging.getLogger("foremast.rollout")

STRATEGIES = ("canary", "rollingupdate")
ALGORITHMS = ("holt_winters", "exponential_smoothing", "double_exponential_smoothing", "moving_average",
              "moving_average_all", "seasonal_decompose")
HB = 16  # forecast offsets kept per row (kernels.HALF_HB): horizons 1..16 of the current window
_SPLIT = ("namespace_pod_caller:", "namespace_app_caller:", "namespace_app_caller_per_pod:",
          "namespace_pod_uri:", "namespace_app_uri:", "namespace_app_uri_per_pod:")
_REGEX_META = re.compile(r"[*+?()\[\]{}^$\\]")


@dataclass
class RolloutSeries:
    """One (job, metric alias): a row of the rollout table."""
    alias: str
    hkey: Key                       # 7-day history series (endpoint, metric, namespace, app)
    fam: Tuple[str, str]            # (endpoint, pod metric) of the current window
    namespace: str
    cur_pods: Tuple[str, ...]
    base_pods: Tuple[str, ...]
    cur_start: float
    cur_n: int
    base_start: float
    base_n: int
    hist_end: float
    base_fam: Tuple[str, str] = ("", "")  # (endpoint, pod metric) of the baseline window (may be another cluster)


@dataclass
class RolloutPlan:
    doc_id: str
    app: Tuple[str, str]
    end_ts: float
    series: List[RolloutSeries]
    doc: Dict = field(default_factory=dict)
    rows: List[int] = field(default_factory=list)


def _pods_of(sel) -> Optional[Tuple[str, Tuple[str, ...]]]:
    """(namespace, pods) of ``<m>{namespace="ns", pod="a"}`` / ``pod=~"a|b"``."""
    ns, pods = None, None
    for label, op, val in sel.matchers:
        if label == "namespace" and op == "=":
            ns = val
        elif label == "pod" and op == "=":
            pods = (val,)
        elif label == "pod" and op == "=~":
            if _REGEX_META.search(val):
                return None
            pods = tuple(p for p in val.split("|") if p)
        else:
            return None
    if ns is None or not pods:
        return None
    return ns, tuple(sorted(set(pods)))


_SIMPLE_SEL = re.compile(r'^([a-zA-Z_:][a-zA-Z0-9_:]*)\{((?:[a-zA-Z_][a-zA-Z0-9_]*(?:=~|=)"[^"\\]*",?)*)\}$')


class _Sel:
    __slots__ = ("name", "matchers")

    def __init__(self, name, matchers):
        self.name, self.matchers = name, matchers


def _selector(q: str):
    """The plain selectors barrelman writes (``name{l="v",l=~"a|b"}``, no
    escapes) split without the general PromQL matcher regex; anything else
    goes through :func:`parse_selector`."""
    m = _SIMPLE_SEL.match(q)
    if m is None:
        return parse_selector(q)
    out = []
    for part in m.group(2).split('",'):
        if not part:
            continue
        label, _, rest = part.partition("=")
        op = "=~" if rest.startswith("~") else "="
        out.append((label, op, rest[2 if op == "=~" else 1:].rstrip('"')))
    return _Sel(m.group(1), tuple(out))


def _grid(url: str) -> Tuple[str, object, float, float, float]:
    """(endpoint, selector, start, end, step) of a flattened Prometheus
    ``query_range`` URL (``prometheushelper.go:12-27`` shape: four parameters,
    only the query percent-encoded); other shapes take the general parser."""
    ep, sep, qs = url.partition("query_range?")
    fields = dict(kv.partition("=")[::2] for kv in qs.split("&")) if sep else {}
    if set(fields) != {"query", "start", "end", "step"}:
        p = urls.parse_prometheus_url(url)
        return ep, parse_selector(str(p["query"])), float(p["start"]), float(p["end"]), float(p["step"])
    return (ep, _selector(_unquote(fields["query"])), float(fields["start"]), float(fields["end"]),
            float(fields["step"]))


_ESC = (("%3A", ":"), ("%7B", "{"), ("%7D", "}"), ("%3D", "="), ("%22", '"'), ("%2C", ","), ("%7C", "|"),
        ("%7E", "~"), ("%2F", "/"))


def _unquote(q: str) -> str:
    """Percent-decoding of a selector: the escapes a PromQL selector of k8s
    names produces are replaced directly (C string ops); any other escape
    takes ``urllib.parse.unquote``."""
    if "%" not in q:
        return q
    for a, b in _ESC:
        q = q.replace(a, b)
    return unquote(q) if "%" in q else q


_PLANS: "OrderedDict[Tuple[str, str], Optional[RolloutPlan]]" = OrderedDict()


def plan_rollout(doc: Dict, cfg: BrainConfig, step: float = 60.0, window_cols: int = 11) -> Optional[RolloutPlan]:
    """The rollout-table plan of a job, or None when the resident engine cannot
    key it.  Memoised per job id (content-addressed: the request, hence the
    plan, never changes), because the claim filters of several engines ask
    for the same documents."""
    if cfg.algorithm not in ALGORITHMS:
        return None
    ck = (doc.get("id", ""), step, window_cols)
    if ck in _PLANS:
        _PLANS.move_to_end(ck)
        return _PLANS[ck]
    plan = _plan(doc, step, window_cols)
    _PLANS[ck] = plan
    if len(_PLANS) > 65536:
        _PLANS.popitem(last=False)
    return plan


def _plan(doc, step, window_cols) -> Optional[RolloutPlan]:
    if (doc.get("strategy") or "").lower() not in STRATEGIES:
        return None
    try:
        cur = urls.parse_config(doc.get("currentConfig", ""))
        base = urls.parse_config(doc.get("baselineConfig", ""))
        hist = urls.parse_config(doc.get("historicalConfig", ""))
        stores = [v for k in ("currentMetricStore", "baselineMetricStore", "historicalMetricStore")
                  for v in urls.parse_config(doc.get(k, "")).values()]
    except urls.ConfigError:
        return None
    if not cur or any(s and s != r.DATASOURCE_PROMETHEUS for s in stores):
        return None
    try:
        end_ts = parse_rfc3339(doc.get("endTime", "")).timestamp()
    except TimeFormatError:
        return None
    out, app = [], None
    for alias in sorted(cur):
        if alias not in hist:
            return None
        try:
            ep_h, sel_h, _hs, h_end, h_step = _grid(hist[alias])
            ep_c, sel_c, c_start, c_end, c_step = _grid(cur[alias])
        except (urls.ConfigError, SelectorError, KeyError, ValueError):
            return None
        lab = {k: v for k, op, v in sel_h.matchers if op == "="}
        if (len(sel_h.matchers) != 2 or set(lab) != {"namespace", "app"} or not sel_h.name or not sel_c.name
                or sel_h.name.startswith(_SPLIT) or sel_c.name.startswith(_SPLIT)
                or h_step != step or c_step != step or ep_c != ep_h):
            return None
        pc = _pods_of(sel_c)
        if pc is None or pc[0] != lab["namespace"]:
            return None
        b_pods, b_start, b_n = (), 0.0, 0
        if alias in base:
            try:
                ep_b, sel_b, b_start, b_end, b_step = _grid(base[alias])
            except (urls.ConfigError, SelectorError, KeyError, ValueError):
                return None
            pb = _pods_of(sel_b)
            # the baseline may live in another cluster (its own Prometheus): multi-cluster canary
            if pb is None or sel_b.name != sel_c.name or b_step != step or pb[0] != pc[0]:
                return None
            b_pods, b_n = pb[1], min(window_cols, int(round((b_end - b_start) / step)) + 1)
            if b_n > 0 and int(round((b_end - b_start) / step)) + 1 > window_cols:
                b_start = b_end - (window_cols - 1) * step  # the newest window_cols points
        app = app or (lab["namespace"], lab["app"])
        out.append(RolloutSeries(
            alias=alias, hkey=(ep_h, sel_h.name, lab["namespace"], lab["app"]), fam=(ep_c, sel_c.name),
            namespace=pc[0], cur_pods=pc[1], base_pods=b_pods, cur_start=c_start,
            cur_n=max(0, min(window_cols, int(round((c_end - c_start) / step)) + 1)),
            base_start=b_start, base_n=b_n, hist_end=h_end,
            base_fam=(ep_b, sel_b.name) if alias in base else ("", "")))
    return RolloutPlan(doc_id=doc["id"], app=app, end_ts=end_ts, series=out, doc=doc)


def is_rollout_keyable(doc: Dict, cfg: BrainConfig) -> bool:
    return plan_rollout(doc, cfg) is not None


class PodSlots:
    """``(namespace, pod)`` -> slot: the row of a pod in each metric family's part
    of the per-tick decode block.  Slots are reference counted by the jobs
    watching the pod (two jobs on one pod share it); key hashes are computed
    once per pod, so the per-family native key indexes are rebuilt from arrays
    when the pod set changes, without touching Python strings."""

    def __init__(self, cap: int = 1024) -> None:
        self.index: Dict[Tuple[str, str], int] = {}
        self.cap = int(cap)
        self.refs = np.zeros(self.cap, dtype=np.int32)
        self.hash = np.zeros(self.cap, dtype=np.uint64)
        self.free: List[int] = list(range(self.cap - 1, -1, -1))
        self.version = 0   # bumps when the pod set changes
        self.added = 0     # bumps when a pod gets a slot (key indexes rebuild)
        self.grown = 0     # bumps when cap grows (every src row moves)

    def acquire(self, keys: List[Tuple[str, str]]) -> np.ndarray:
        new = list(dict.fromkeys(k for k in keys if k not in self.index))
        if new:
            while len(self.free) < len(new):
                old = self.cap
                self.cap *= 2
                self.refs = np.concatenate([self.refs, np.zeros(old, dtype=np.int32)])
                self.hash = np.concatenate([self.hash, np.zeros(old, dtype=np.uint64)])
                self.free = list(range(self.cap - 1, old - 1, -1)) + self.free
                self.grown += 1
            hs = native.key_hashes([k[0] for k in new], [k[1] for k in new])
            for k, h in zip(new, hs):
                slot = self.free.pop()
                self.index[k] = slot
                self.hash[slot] = h
            self.version += 1
            self.added += 1
        slots = np.fromiter((self.index[k] for k in keys), dtype=np.int64, count=len(keys))
        np.add.at(self.refs, slots, 1)
        return slots

    def release(self, keys: List[Tuple[str, str]]) -> None:
        for k in keys:
            slot = self.index.get(k)
            if slot is None:
                continue
            self.refs[slot] -= 1
            if self.refs[slot] <= 0:
                self.refs[slot] = 0
                del self.index[k]
                self.free.append(slot)
                self.version += 1

    def live(self) -> np.ndarray:
        return np.fromiter(self.index.values(), dtype=np.int64, count=len(self.index))


class RolloutMonitor:
    def __init__(self, store: JobStore, cfg: Optional[BrainConfig] = None, prom=None, device=None,
                 worker_id: str = "rollout-0", metrics: Optional[BrainMetrics] = None, step: float = 60.0,
                 window: int = 10, pods: int = 5, clock=time.time, owns: Optional[Callable[[Dict], bool]] = None,
                 history: Optional[ResidentHistory] = None, ring_len: Optional[int] = None,
                 min_capacity: int = 64, decode_threads: int = 8, apps_per_query: int = 256,
                 claim_limit: int = 100_000) -> None:
        from ..promql.client import PromClient
        self.store = store
        self.cfg = cfg or BrainConfig.from_env()
        self.prom = prom or PromClient()
        self.device = torch.device(device) if device is not None else (
            torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu"))
        self.gpu = self.device.type == "cuda"
        self.worker_id = worker_id
        self.metrics = metrics or BrainMetrics()
        self.step, self.clock, self.owns = float(step), clock, owns
        self.Wc = int(window) + 1            # [start + step, start + (W + 1) step] (metricsquery.go:52-64)
        self.P = max(1, int(pods))
        self.season = max(2, int(round(86400.0 / self.step)))
        self.m_detect = max(self.season, HB)
        self.decode_threads = max(1, int(decode_threads))
        self.apps_per_query = max(1, int(apps_per_query))
        self.claim_limit = claim_limit
        self.history = history or ResidentHistory(self.prom, self.device, ring_len or self.cfg.ring_len, self.step,
                                                  clock=clock, decode_threads=decode_threads,
                                                  apps_per_query=apps_per_query)
        self.min_capacity = max(1, int(min_capacity))
        self.jobs: Dict[str, RolloutPlan] = {}        # admitted (rows assigned)
        self.waiting: Dict[str, RolloutPlan] = {}     # claimed, history not resident yet
        self._ends: List[Tuple[float, str]] = []      # (end_ts, job) heap of admitted jobs
        self.row_plan: List[Optional[Tuple[str, int]]] = []   # row -> (job id, series index)
        self.apps: Dict[Tuple[str, str], int] = {}
        self.roster_version = 0
        self.t_cur = 0.0                               # newest minute ingested into the windows
        self.ticks = 0
        self.tick_queries = 0
        self.admitted = 0
        self.cap = 0
        self.slots = PodSlots()
        self.fams: Dict[Tuple[str, str], int] = {}     # pod metric family -> index in the decode block
        self._tables = None                            # (slots.version, cap, fam tables)
        self._srcmap_dirty = True
        self._blocks: Dict[Tuple[int, int], List[torch.Tensor]] = {}
        self._block_i = 0
        # cluster-affine ingest (parallel/affine.py): windows of another rank's clusters are
        # requested at admission and delivered by that rank in the tick's lockstep exchange
        self.router = None
        self._remote: List[Tuple[str, Tuple[str, str], float, int, List]] = []
        self.timings: Dict[str, float] = {}
        self._bands: Tuple[np.ndarray, np.ndarray, np.ndarray] = (np.zeros(0), np.zeros(0), np.zeros(0))
        self._last_anom: Dict[int, float] = {}
        self._apps_dirty = False
        self._app_refs: Dict[Tuple[str, str], int] = {}
        self._app_names: List[Optional[Tuple[str, str]]] = []   # app index -> name (None: free index)
        self._app_free: List[int] = []
        self._app_new: List[Tuple[Tuple[str, str], List[int]]] = []
        self._app_gone: List[Tuple[str, str]] = []
        self._n_live = 0
        self._build_grid()
        self.anomalies = None
        self.metrics.add_band_source(f"rollout:{worker_id}", self._band_rows)

    # ------------------------------------------------------------------ model grid
    def _build_grid(self) -> None:
        """One table of (alpha, beta, gamma) rows for every smoothing family: a
        row's fitted grid point indexes it (h-step variance; unused axes are 0,
        so the Holt-Winters closed form is exact for ES / DES too)."""
        cfg = self.cfg
        parts, self.grid_off = [], {}
        off = 0
        for mode in (sm_ref.MODE_HW, sm_ref.MODE_ES, sm_ref.MODE_DES):
            g = sm_ref.make_grid(mode, cfg.hw_alpha, cfg.hw_beta, cfg.hw_gamma)
            self.grid_off[mode] = off
            off += g.shape[0]
            parts.append(g)
        self.grids = {mode: p.to(self.device).contiguous() for mode, p in zip(self.grid_off, parts)}
        self.grid_all = torch.cat(parts).to(self.device).contiguous()

    # ------------------------------------------------------------------ storage
    def _alloc(self, cap: int) -> None:
        dev, C = self.device, self.P * self.Wc
        f32 = dict(dtype=torch.float32, device=dev)
        old = getattr(self, "win", None)
        n = self.cap
        old_app_id = getattr(self, "app_id", None)
        new = {
            "win": torch.full((cap, C), float("nan"), **f32),
            "base": torch.full((cap, C), float("nan"), **f32),
            "hz": torch.ones((cap, C), dtype=torch.int32, device=dev),
            "threshold": torch.full((cap,), self.cfg.threshold, **f32),
            "bound": torch.full((cap,), self.cfg.bound, dtype=torch.int8, device=dev),
            "min_lower": torch.zeros(cap, **f32),
            "app_id": torch.zeros(cap, dtype=torch.int32, device=dev),
            "start_min": torch.zeros(cap, dtype=torch.int32, device=dev),
        }
        st = {k: torch.zeros(cap, **f32) for k in ("level", "trend", "sigma", "nvalid")}
        st["best"] = torch.full((cap,), -1, dtype=torch.int32, device=dev)
        st["season_hb"] = torch.zeros((cap, HB), **f32)
        if old is not None:
            for k, t in new.items():
                t[:n].copy_(getattr(self, k))
            for k, t in st.items():
                t[:n].copy_(self.state[k])
        for k, t in new.items():
            setattr(self, k, t)
        self.state = st
        self.out: Dict[str, torch.Tensor] = {}
        self.pw_out: Dict[str, torch.Tensor] = {}
        self.app_stats = torch.zeros((max(1, len(self._app_names)), 2), dtype=torch.int32, device=dev)
        if n:  # rows keep their app index across growth
            self.app_id[:n].copy_(old_app_id)
        self.row_plan.extend([None] * (cap - len(self.row_plan)))
        self.model_ok = np.concatenate([getattr(self, "model_ok", np.zeros(0, bool)), np.zeros(cap - n, bool)])
        self.row_fam = np.concatenate([getattr(self, "row_fam", np.zeros(0, np.int64)), np.full(cap - n, -1)])
        self.row_slot = np.concatenate([getattr(self, "row_slot", np.zeros((0, self.P), np.int64)),
                                        np.full((cap - n, self.P), -1)])
        self._srcmap_dirty = True
        self.cap = cap
        if self.gpu:
            from ..ops import kernels as K
            self.anomalies = K.AnomalyBuffer(max(1024, 4 * cap), dev)

    def _free_rows(self, rows: List[int]) -> None:
        if not rows:
            return
        idx = torch.tensor(rows, dtype=torch.long, device=self.device)
        self.win.index_fill_(0, idx, float("nan"))
        self.base.index_fill_(0, idx, float("nan"))
        self.app_id.index_fill_(0, idx, 0)
        for row in rows:
            self.row_plan[row] = None
            self.model_ok[row] = False
        self.row_fam[rows] = -1
        self.row_slot[rows] = -1
        self._n_live -= len(rows)
        self._srcmap_dirty = True

    def _take_rows(self, n: int) -> List[int]:
        free = [i for i, p in enumerate(self.row_plan) if p is None]
        if len(free) < n:
            used = self.cap - len(free)
            cap = max(self.min_capacity, self.cap or 1)
            while cap < used + n:
                cap *= 2
            self._alloc(cap)
            free = [i for i, p in enumerate(self.row_plan) if p is None]
        return free[:n]

    @property
    def n_live(self) -> int:
        return self._n_live

    # ------------------------------------------------------------------ membership
    def owns_affine(self, d) -> bool:
        """Cluster-affine mode: a job belongs to the rank that scrapes the cluster
        of its new pods (its history and current windows are then local)."""
        p = plan_rollout(d, self.cfg, self.step, self.Wc)
        return p is not None and self.router.local(p.series[0].fam[0])

    def _claimable(self, d) -> bool:
        return plan_rollout(d, self.cfg, self.step, self.Wc) is not None and (self.owns is None or self.owns(d))

    def sync(self, steal_from=None) -> int:
        """Lease new keyable rollout jobs (that this rank owns)."""
        now = self.clock()
        docs = self.store.claim(self.worker_id, now=now, max_stuck_s=self.cfg.max_stuck_seconds,
                                limit=self.claim_limit, only=self._claimable, steal_from=steal_from)
        for d in docs:
            p = plan_rollout(d, self.cfg, self.step, self.Wc)
            if p is None or d["id"] in self.jobs or d["id"] in self.waiting:
                continue
            p.doc = d
            self.waiting[d["id"]] = p
            self.history.want([s.hkey for s in p.series], now)
        return len(docs)

    def release(self, pred: Callable[[Dict], bool]) -> int:
        """Hand back the leases of jobs matching ``pred`` (their app moved to
        another rank); their rows are freed at once."""
        now = self.clock()
        back = []
        for jid, p in list(self.jobs.items()) + list(self.waiting.items()):
            if pred(p.doc):
                back.append((jid, {"status": r.ST_REPROGRESS, "claimed_by": "", "not_before": 0.0}))
                self._drop(jid, now)
        if back:
            self.store.update_many(back, expect_claimed_by=self.worker_id)
        return len(back)

    def _drop(self, jid: str, now: float) -> None:
        p = self.jobs.pop(jid, None) or self.waiting.pop(jid, None)
        if p is None:
            return
        self.history.unwant([s.hkey for s in p.series], now)
        self._free_rows(p.rows)
        if p.rows:
            self._app_ref(p, -1)
            self.slots.release(self._job_pods(p))
        p.rows = []

    def _refresh_apps(self) -> None:
        """Apply the app-roster changes of the last admissions / verdicts.  App
        indices are stable (a freed index is reused by a later app), so a job
        finishing never renumbers the other rows; called only before scoring,
        so the roster :meth:`app_table` reports is the one the last tick's
        counters were accumulated under."""
        if not self._apps_dirty:
            return
        for a in self._app_gone:
            if self._app_refs.get(a, 0) <= 0 and a in self.apps:
                i = self.apps.pop(a)
                self._app_names[i] = None
                self._app_free.append(i)
        self._app_gone = []
        for a, rows in self._app_new:
            i = self.apps.get(a)
            if i is None:
                i = self._app_free.pop() if self._app_free else len(self._app_names)
                if i == len(self._app_names):
                    self._app_names.append(a)
                else:
                    self._app_names[i] = a
                self.apps[a] = i
            if rows:
                self.app_id[torch.tensor(rows, dtype=torch.long, device=self.device)] = i
        self._app_new = []
        if self.cap and self.app_stats.shape[0] < max(1, len(self._app_names)):
            cap = self.app_stats.shape[0]
            while cap < len(self._app_names):
                cap *= 2
            self.app_stats = torch.zeros((cap, 2), dtype=torch.int32, device=self.device)
        self.roster_version += 1
        self._apps_dirty = False

    def _app_ref(self, p: RolloutPlan, delta: int) -> None:
        n = self._app_refs.get(p.app, 0) + delta
        self._app_refs[p.app] = n
        if delta > 0:
            self._app_new.append((p.app, list(p.rows)))
        elif n <= 0:
            self._app_refs.pop(p.app, None)
            self._app_gone.append(p.app)
        self._apps_dirty = True

    # ------------------------------------------------------------------ admission
    async def _admit(self, now: float) -> int:
        ready = [p for p in self.waiting.values() if all(self.history.ready(s.hkey) for s in p.series)]
        if not ready:
            return 0
        t0 = time.perf_counter()
        n_rows = sum(len(p.series) for p in ready)
        rows = self._take_rows(n_rows)
        it = iter(rows)
        items: List[Tuple[int, RolloutSeries]] = []
        for p in ready:
            del self.waiting[p.doc_id]
            p.rows = [next(it) for _ in p.series]
            for k, (row, s) in enumerate(zip(p.rows, p.series)):
                self.row_plan[row] = (p.doc_id, k)
                items.append((row, s))
            self.jobs[p.doc_id] = p
            self._n_live += len(p.series)
            heapq.heappush(self._ends, (p.end_ts, p.doc_id))
        self._set_row_params(items)
        self._assign_slots(ready)
        self._fit(items)
        await self._load_windows(items)
        self.admitted += len(ready)
        for p in ready:
            self._app_ref(p, +1)
        self.timings["admit_ms"] = (time.perf_counter() - t0) * 1e3
        return len(ready)

    def _set_row_params(self, items: List[Tuple[int, RolloutSeries]]) -> None:
        dev = self.device
        rows = torch.tensor([row for row, _ in items], dtype=torch.long, device=dev)
        f = lambda xs, dt: torch.tensor(xs, dtype=dt, device=dev)  # noqa: E731
        th = {}
        for _, s in items:
            if (s.alias, s.hkey[1]) not in th:
                th[(s.alias, s.hkey[1])] = self.cfg.for_metric(s.alias, s.hkey[1])
        ths = [th[(s.alias, s.hkey[1])] for _, s in items]
        self.threshold[rows] = f([t.threshold for t in ths], torch.float32)
        self.bound[rows] = f([t.bound for t in ths], torch.int8)
        self.min_lower[rows] = f([t.min_lower_bound for t in ths], torch.float32)
        self.start_min[rows] = f([int(round(s.cur_start / self.step)) for _, s in items], torch.int32)
        self.win[rows] = float("nan")
        self.base[rows] = float("nan")

    def _fit(self, items: List[Tuple[int, RolloutSeries]]) -> None:
        """Fit every admitted row's model on its history ending at the job's
        start (grouped by how many of the ring's newest points that drops) and
        store the forecast state + per-column horizons."""
        hist = self.history
        groups: Dict[int, List[Tuple[int, RolloutSeries]]] = {}
        for row, s in items:
            drop = int(round((hist.t_last - s.hist_end) / self.step))
            groups.setdefault(max(0, drop), []).append((row, s))
        Wc = self.Wc
        for drop, grp in groups.items():
            t_fit = hist.t_last - drop * self.step
            rows = [row for row, _ in grp]
            data, head, length = hist.gather([hist.rows[s.hkey] for _, s in grp], drop)
            st = self._fit_state(data, head, length)
            idx = torch.tensor(rows, dtype=torch.long, device=self.device)
            for k, v in st.items():
                self.state[k][idx] = v.to(self.state[k].dtype)
            self.model_ok[rows] = (st["nvalid"] >= self.cfg.min_historical_points).cpu().numpy()
            off = np.array([int(round((s.cur_start - t_fit) / self.step)) for _, s in grp], dtype=np.int64)
            hz = off[:, None] + np.tile(np.arange(Wc), self.P)[None, :]
            self.hz[idx] = torch.from_numpy(np.clip(hz, 1, 1 << 20).astype(np.int32)).to(self.device)

    def _algo_for(self, length: int) -> str:
        algo, m = self.cfg.algorithm, self.season
        if algo == "holt_winters" and length < 2 * m:
            algo = "double_exponential_smoothing"
        if algo == "seasonal_decompose" and length < 2 * m + 1:
            algo = "moving_average_all"
        return algo

    def _fit_state(self, data: torch.Tensor, head: int, length: int) -> Dict[str, torch.Tensor]:
        """Forecast state of each row's model on the logical window ``[head, head
        + length)`` of ``data``: level, trend, season_hb (forecast offsets of
        horizons 1..16), sigma, nvalid, best (row of ``grid_all``, -1 = no
        h-step variance)."""
        algo = self._algo_for(length)
        k, dev, cfg = data.shape[0], self.device, self.cfg
        hs = torch.arange(1, HB + 1, dtype=torch.int32, device=dev)
        mode = sm_ref.MODE_BY_NAME.get(algo)
        if self.gpu:
            from ..ops import kernels as K
            spec = K.DetectSpec(horizons=hs, threshold=torch.ones(k, device=dev),
                                bound=torch.full((k,), 3, dtype=torch.int8, device=dev),
                                min_lower=torch.zeros(k, device=dev), max_horizon=HB,
                                horizon_variance=False)
            if mode is not None:
                m = self.season if mode == sm_ref.MODE_HW else 1
                out = K.smoothing_fit(data, head, length, mode, m, self.grids[mode], spec, defer_detect=True)
                if K.last_detect_deferred:
                    st = {"level": out["level"], "trend": out["trend"], "sigma": out["sigma"],
                          "nvalid": out["nvalid"], "season_hb": out["season_hb"],
                          "best": out["best"] + self.grid_off[mode]}
                    if mode == sm_ref.MODE_HW:  # season_hb holds the phases of horizons 1..16 after the fit end
                        return st
                    st["season_hb"] = torch.zeros((k, HB), device=dev)
                    return st
                # geometry without the deferred path: the epilogue's forecast of horizons 1..16
                out = K.smoothing_fit(data, head, length, mode, m, self.grids[mode], spec)
                cnt = K.window_stats(data, head, length, spec)["count_hist"]
                return {"level": out["level"], "trend": out["trend"], "sigma": out["sigma"], "nvalid": cnt,
                        "season_hb": out["forecast"] - out["level"][:, None] - hs[None, :] * out["trend"][:, None],
                        "best": out["best"] + self.grid_off[mode]}
            if algo == "seasonal_decompose":
                out = K.decompose_score(data, head, length, self.season, spec)
                return {"level": out["level"], "trend": out["slope"], "sigma": out["sigma"], "nvalid": out["nvalid"],
                        "season_hb": out["forecast"] - out["level"][:, None] - hs[None, :] * out["slope"][:, None],
                        "best": torch.full((k,), -1, dtype=torch.int32, device=dev)}
            h0, ln = head, length
            if algo == "moving_average" and cfg.ma_window < length:
                h0, ln = (head + length - cfg.ma_window) % data.shape[1], cfg.ma_window
            out = K.window_stats(data, h0, ln, spec)
            return {"level": out["mean"], "trend": torch.zeros(k, device=dev), "sigma": out["std"],
                    "nvalid": out["count_hist"], "season_hb": torch.zeros((k, HB), device=dev),
                    "best": torch.full((k,), -1, dtype=torch.int32, device=dev)}
        # CPU: the PyTorch reference models
        R = data.shape[1]
        idx = (torch.arange(length) + head) % R
        y = data.index_select(1, idx).float()
        hsl = hs.long()
        if mode is not None:
            fit = sm_ref.fit_smoothing(y, mode, self.grids[mode].cpu(), m=self.season if mode == sm_ref.MODE_HW else 1)
            f = sm_ref.forecast(fit, hsl)
            return {"level": fit.level, "trend": fit.trend, "sigma": fit.sigma, "nvalid": fit.n_valid.float(),
                    "season_hb": f - fit.level[:, None] - hsl[None, :] * fit.trend[:, None],
                    "best": fit.best.int() + self.grid_off[mode]}
        if algo == "seasonal_decompose":
            fc = dec_ref.decompose_forecast(y, self.season)
            f = dec_ref.forecast_decomposition(fc, hsl)
            return {"level": fc.level, "trend": fc.slope, "sigma": fc.sigma, "nvalid": fc.n_valid.float(),
                    "season_hb": f - fc.level[:, None] - hsl[None, :] * fc.slope[:, None],
                    "best": torch.full((k,), -1, dtype=torch.int32)}
        ws = ma_ref.window_stats(y, cfg.ma_window if algo == "moving_average" else None)
        return {"level": ws.mean, "trend": torch.zeros(k), "sigma": ws.std, "nvalid": ws.count.float(),
                "season_hb": torch.zeros((k, HB)), "best": torch.full((k,), -1, dtype=torch.int32)}

    @staticmethod
    def _job_pods(p: RolloutPlan) -> List[Tuple[str, str]]:
        """The (namespace, pod) keys a job holds slots for (current pods, once per job)."""
        return list(dict.fromkeys((s.namespace, pod) for s in p.series for pod in s.cur_pods))

    def _fam(self, fam: Tuple[str, str]) -> int:
        fi = self.fams.get(fam)
        if fi is None:
            fi = self.fams[fam] = len(self.fams)
            self._tables = None
        return fi

    def _assign_slots(self, plans: List[RolloutPlan]) -> None:
        P = self.P
        for p in plans:
            keys = self._job_pods(p)
            slots = dict(zip(keys, self.slots.acquire(keys).tolist()))
            for row, s in zip(p.rows, p.series):
                self.row_fam[row] = self._fam(s.fam)
                pods = s.cur_pods[:P]
                self.row_slot[row, :len(pods)] = [slots[(s.namespace, pod)] for pod in pods]
                self.row_slot[row, len(pods):] = -1
        self._srcmap_dirty = True

    def _srcmap(self) -> torch.Tensor:
        """Device ``[cap * P]`` src row of every (row, pod): family x slot cap + slot."""
        if self._srcmap_dirty or getattr(self, "_srcmap_grown", -1) != self.slots.grown:
            fam = self.row_fam[:, None]
            m = np.where((self.row_slot >= 0) & (fam >= 0), fam * self.slots.cap + self.row_slot, -1)
            self._srcmap_t = torch.from_numpy(m.astype(np.int32).reshape(-1)).to(self.device)
            self._srcmap_dirty = False
            self._srcmap_grown = self.slots.grown
        return self._srcmap_t

    def _key_tables(self) -> Dict[Tuple[str, str], native.KeyTable]:
        """Per pod family: native (namespace, pod) -> src row index over the live slots.

        Rebuilt only when a pod gets a slot (or the slots grow), not when pods leave: a
        released pod's key still maps to its old slot until that slot is reused, and the
        points decoded there are never scattered (no live series reads a free slot).  So
        the ticks on which jobs finish do not pay an index rebuild (~10 ms at 100k keys) in
        their decode."""
        key = (self.slots.added, self.slots.cap, len(self.fams))
        if self._tables is None or self._tables[0] != key:
            live = self.slots.live()
            h = self.slots.hash[live]
            used = {f for f in self.row_fam.tolist() if f >= 0}
            tabs = {fam: native.KeyTable.indexed(h, fi * self.slots.cap + live, "namespace", "pod")
                    for fam, fi in self.fams.items() if fi in used}
            for t in tabs.values():
                t.index  # build the native index now, not inside the first decode
            self._tables = (key, tabs)
        return self._tables[1]

    async def _load_windows(self, items: List[Tuple[int, RolloutSeries]]) -> None:
        """Baseline windows (fixed: ``[start - W, start]``) and any current points
        that already exist (a job claimed late), per (kind, window start): one
        query per pod family and group of jobs, every body decoded through one
        key index over the group's pods, then gathered into the rows."""
        t_last = self.history.t_last
        # (kind, window start, points) -> [(row, series, pods, family)]
        groups: Dict[Tuple[str, float, int], List[Tuple[int, RolloutSeries, Tuple[str, ...], Tuple[str, str]]]] = {}
        for row, s in items:
            if s.base_pods and s.base_n > 0:
                groups.setdefault(("base", s.base_start, s.base_n), []).append((row, s, s.base_pods, s.base_fam))
            if s.cur_n > 0 and s.cur_start <= t_last:
                n = min(s.cur_n, int(round((t_last - s.cur_start) / self.step)) + 1)
                groups.setdefault(("win", s.cur_start, n), []).append((row, s, s.cur_pods, s.fam))
        P, Wc = self.P, self.Wc
        if self.router is not None:  # windows of other ranks' clusters: requested, not fetched
            for (dst, start, n), grp in list(groups.items()):
                remote = [g for g in grp if not self.router.local(g[3][0])]
                if not remote:
                    continue
                groups[(dst, start, n)] = [g for g in grp if self.router.local(g[3][0])]
                for f in dict.fromkeys(g[3] for g in remote):
                    part = [(row, s, ps) for row, s, ps, fam in remote if fam == f]
                    pods = list(dict.fromkeys((s.namespace, pod) for _, s, ps in part for pod in ps[:P]))
                    self._remote.append((dst, f, start, n, part, pods))
            groups = {k: v for k, v in groups.items() if v}
        for (dst, start, n), grp in groups.items():
            pods = list(dict.fromkeys((s.namespace, pod) for _, s, ps, _f in grp for pod in ps[:P]))
            local = {k: i for i, k in enumerate(pods)}
            fams = list(dict.fromkeys(f for _, _, _, f in grp))
            fidx = {f: i for i, f in enumerate(fams)}
            nl = len(pods)
            hs = native.key_hashes([k[0] for k in pods], [k[1] for k in pods])
            block_t = torch.full((len(fams) * nl, Wc), float("nan"), dtype=torch.float32)
            if self.gpu:
                block_t = block_t.pin_memory()
            tables = {f: native.KeyTable.indexed(hs, fidx[f] * nl + np.arange(nl), "namespace", "pod") for f in fams}
            reqs, tabs = [], []
            for f in fams:
                rows_f = [(s, ps) for _, s, ps, ff in grp if ff == f]
                for g in range(0, len(rows_f), self.apps_per_query):
                    part = rows_f[g:g + self.apps_per_query]
                    sel = (f'{f[1]}{{namespace=~"{re_alt({s.namespace for s, _ in part})}",'
                           f'pod=~"{re_alt({pod for _, ps in part for pod in ps[:P]})}"}}')
                    reqs.append((range_url(f[0], sel, start, n, self.step), start, n, 0))
                    tabs.append(tables[f])
            ok = await fetch_decode(self.prom, reqs, tabs, block_t.numpy(), self.step, self.decode_threads)
            if not all(ok):
                log.warning("%d of %d window queries failed (%s from %d)", ok.count(False), len(ok), dst, start)
            gidx = np.full((len(grp), P), -1, dtype=np.int64)
            for i, (_, s, ps, f) in enumerate(grp):
                fo = fidx[f] * nl
                for p, pod in enumerate(ps[:P]):
                    gidx[i, p] = fo + local[(s.namespace, pod)]
            blk = block_t.to(self.device, non_blocking=True)
            gi = torch.from_numpy(gidx).to(self.device)
            vals = blk[gi.clamp(min=0)]                       # [k, P, Wc]
            vals = torch.where((gi >= 0)[:, :, None], vals, torch.full_like(vals, float("nan")))
            rows = torch.tensor([row for row, _, _, _ in grp], dtype=torch.long, device=self.device)
            (self.base if dst == "base" else self.win).index_copy_(0, rows, vals.reshape(len(grp), P * Wc))

    async def _serve_windows(self, requests) -> List[np.ndarray]:
        """Fetch + decode window requests of this rank's clusters (cluster-affine mode)."""
        out = []
        for fam, start, n, pods in requests:
            hs = native.key_hashes([k[0] for k in pods], [k[1] for k in pods])
            table = native.KeyTable.indexed(hs, np.arange(len(pods)), "namespace", "pod")
            buf = np.full((len(pods), n), np.nan, dtype=np.float32)
            reqs = []
            for g in range(0, len(pods), self.apps_per_query * self.P):
                part = pods[g:g + self.apps_per_query * self.P]
                sel = (f'{fam[1]}{{namespace=~"{re_alt({k[0] for k in part})}",'
                       f'pod=~"{re_alt({k[1] for k in part})}"}}')
                reqs.append((range_url(fam[0], sel, start, n, self.step), start, n, 0))
            ok = await fetch_decode(self.prom, reqs, [table] * len(reqs), buf, self.step, self.decode_threads)
            if not all(ok):
                log.warning("served window request %s from %d: %d queries failed", fam[1], start, ok.count(False))
            out.append(buf)
        return out

    async def _route(self) -> None:
        """Cluster-affine lockstep exchange of this tick's remote window requests."""
        mine, self._remote = self._remote, []
        vals = await self.router.exchange([(f, st, n, pods) for _dst, f, st, n, _part, pods in mine],
                                          self._serve_windows)
        P, Wc = self.P, self.Wc
        for (dst, f, st, n, part, pods), v in zip(mine, vals):
            local = {k: i for i, k in enumerate(pods)}
            block = np.full((len(part), P, Wc), np.nan, dtype=np.float32)
            for i, (_row, s, ps) in enumerate(part):
                for p, pod in enumerate(ps[:P]):
                    block[i, p, :n] = v[local[(s.namespace, pod)]]
            rows = torch.tensor([row for row, _, _ in part], dtype=torch.long, device=self.device)
            tgt = self.base if dst == "base" else self.win
            if all(0 <= row < len(self.row_plan) and self.row_plan[row] is not None for row in rows.tolist()):
                tgt.index_copy_(0, rows, torch.from_numpy(block.reshape(len(part), P * Wc)).to(self.device))

    def _tick_block(self, S: int, k: int):
        """NaN-filled pinned decode block of the tick, one of two kept across ticks."""
        bufs = self._blocks.get((S, k))
        if bufs is None:
            bufs = [torch.empty((S, k), dtype=torch.float32) for _ in range(2)]
            if self.gpu:
                bufs = [b.pin_memory() for b in bufs]
            self._blocks = {(S, k): bufs}
        self._block_i ^= 1
        t = bufs[self._block_i]
        a = t.numpy()
        a.fill(np.nan)
        return t, a

    async def _ingest(self, t_new: float) -> None:
        if self.t_cur == 0.0:
            self.t_cur = t_new - self.step  # the first tick fetches the current minute
        k = int(round((t_new - self.t_cur) / self.step))
        if k <= 0 or not self.jobs:
            self.t_cur = max(self.t_cur, t_new)
            return
        k = min(k, 4 * self.Wc)  # behind by more than any window: only the recent minutes matter
        first = t_new - (k - 1) * self.step
        tables = self._key_tables()
        P = self.P
        S = len(self.fams) * self.slots.cap
        block_t, block = self._tick_block(S, k)
        self.timings["points"] = k
        reqs = [(range_url(fam[0], fam[1], first, k, self.step), first, k, 0) for fam in tables]
        self.tick_queries += len(reqs)
        t0 = time.perf_counter()
        ok = await fetch_decode(self.prom, reqs, list(tables.values()), block, self.step, self.decode_threads,
                                timings=self.timings)
        self.timings["decode_ms"] = (time.perf_counter() - t0) * 1e3
        if not all(ok):
            return  # t_cur stays: the next tick fetches these minutes again
        col0 = (int(round(first / self.step)) - self.start_min).to(torch.int32).contiguous()
        srcmap = self._srcmap()
        if self.gpu:
            from ..ops import kernels as K
            K.rollout_scatter(self.win, P, self.Wc, block_t.to(self.device, non_blocking=True), col0, srcmap)
        else:
            win = self.win.view(self.cap, P, self.Wc)
            sm = srcmap.view(self.cap, P).long()
            src = block_t
            for j in range(k):
                c = (col0 + j).long()
                ok_r = ((c >= 0) & (c < self.Wc))[:, None] & (sm >= 0)
                vals = torch.where(ok_r, src[sm.clamp(min=0), j], torch.full(sm.shape, float("nan")))
                keep = ok_r & ~torch.isnan(vals)
                rr, pp = torch.nonzero(keep, as_tuple=True)
                win[rr, pp, c[rr]] = vals[rr, pp]
        self.t_cur = t_new

    def _score(self) -> Dict[str, torch.Tensor]:
        cfg, dev = self.cfg, self.device
        valid = ~torch.isnan(self.win)
        npts = valid.sum(1)
        thr_f, thr_l = det_ref.effective_thresholds(self.threshold, self.bound, npts, cfg.pairwise_scale,
                                                    cfg.window_correction)
        thr_f, thr_l = thr_f.contiguous(), thr_l.contiguous()
        pw_mode = pw_ref.PW_BY_NAME.get(cfg.pairwise_algorithm.upper(), pw_ref.PW_ALL)
        self.app_stats.zero_()
        differs = None
        if self.gpu:
            from ..ops import kernels as K
            if pw_mode != pw_ref.PW_NONE:
                self.pw_out = K.rank_tests(self.base, self.win, pw_mode, cfg.pairwise_threshold, cfg.min_mann_white,
                                           cfg.min_wilcoxon, cfg.min_kruskal, want_pvals=False, out=self.pw_out,
                                           pods=(self.P, self.P), min_friedman=cfg.min_friedman)
                differs = self.pw_out["differs"]
            self.anomalies.reset()
            spec = K.DetectSpec(horizons=self.hz, threshold=thr_f, bound=self.bound, min_lower=self.min_lower,
                                cur=self.win, differs=differs, pw_scale=cfg.pairwise_scale,
                                min_valid=cfg.min_historical_points, want_band=True, app_id=self.app_id,
                                app_stats=self.app_stats, anomalies=self.anomalies, threshold_low=thr_l,
                                pw_min_points=cfg.pairwise_min_points,
                                shift_threshold=cfg.pairwise_shift, shift_min_points=cfg.pairwise_shift_min_points,
                                base_mean=self.pw_out["base_mean"] if differs is not None else None,
                                horizon_variance=cfg.horizon_variance)
            st = dict(self.state)
            st.update(self.out)
            out = K.hw_detect_deferred(st, spec, self.m_detect, self.m_detect,
                                       grid=self.grid_all if cfg.horizon_variance else None)
            self.out = {k: out[k] for k in ("forecast", "upper", "lower", "count", "verdict", "score")}
        else:
            if pw_mode != pw_ref.PW_NONE:
                res = pw_ref.rank_tests(self.base, self.win, pods=(self.P, self.P))
                differs = pw_ref.pairwise_differs(res, pw_mode, cfg.pairwise_threshold, cfg.min_mann_white,
                                                  cfg.min_wilcoxon, cfg.min_kruskal, cfg.min_friedman)
            s = self.state
            h = self.hz.long()
            f = s["level"][:, None] + h * s["trend"][:, None] + s["season_hb"].gather(1, (h.clamp(max=HB) - 1))
            sigma = s["sigma"][:, None].expand_as(f)
            if cfg.horizon_variance:
                best = s["best"].long()
                params = torch.where((best >= 0)[:, None], self.grid_all[best.clamp(min=0)],
                                     torch.zeros((best.shape[0], 3)))
                sigma = sigma * det_ref.horizon_sigma_factor(params, sm_ref.MODE_HW, self.m_detect, h)
            d = det_ref.detect(f, sigma, self.win, thr_f, self.bound, self.min_lower, differs=differs,
                               pairwise_scale=cfg.pairwise_scale, model_ok=s["nvalid"] >= cfg.min_historical_points,
                               threshold_low=thr_l, pw_min_points=cfg.pairwise_min_points,
                               shift_threshold=cfg.pairwise_shift, shift_min_points=cfg.pairwise_shift_min_points,
                               base_mean=torch.nanmean(self.base.float(), 1) if differs is not None else None)
            v = d.verdict.long()
            self.app_stats.index_put_((self.app_id.long(), torch.zeros_like(v)), (v == 1).int(), accumulate=True)
            self.app_stats.index_put_((self.app_id.long(), torch.ones_like(v)), (v >= 0).int(), accumulate=True)
            self.out = {"forecast": f, "upper": d.upper, "lower": d.lower, "count": d.count, "verdict": d.verdict,
                        "score": d.score, "_anomaly": d.anomaly}
        self.out["npts"] = npts
        return self.out

    async def tick(self) -> Dict[str, str]:
        """One tick: heartbeat, history sync, admissions, window ingest, scoring,
        verdicts; returns job -> status written."""
        t_tick = time.perf_counter()
        now = self.clock()
        t_new = float(np.floor(now / self.step) * self.step)
        t0 = time.perf_counter()
        try:
            # inside the guard: a store error on this rank must not skip the lockstep
            # exchange below, or its peers' all_to_all would pair with another collective
            self.store.heartbeat(self.worker_id, now)
            await self.history.sync(now)
            self.timings["history_ms"] = (time.perf_counter() - t0) * 1e3
            await self._admit(now)
        except Exception:  # noqa: BLE001
            if self.router is None:
                raise
            log.exception("rollout data step failed (the affine exchange still runs)")
        if self.router is not None:
            await self._route()  # every rank, every tick (collectives)
        self._refresh_apps()
        written: Dict[str, str] = {}
        if not self.jobs:
            self.t_cur = max(self.t_cur, t_new)
            self._bands = (np.zeros(0), np.zeros(0), np.zeros(0))
            if self.cap:
                self.app_stats.zero_()
            return written
        await self._ingest(t_new)
        t0 = time.perf_counter()
        out = self._score()
        # ONE device->host copy of the per-row results (verdict, points seen, band at the newest column)
        last_c = ((int(round(self.t_cur / self.step)) - self.start_min).clamp(0, self.Wc - 1)).long()
        up = out["upper"].gather(1, last_c[:, None])[:, 0]
        lo = out["lower"].gather(1, last_c[:, None])[:, 0]
        host = torch.stack([out["verdict"].float(), out["npts"].float(), up, lo]).cpu().numpy()
        verdict, npts = host[0].astype(np.int8), host[1]
        if self.gpu:
            a_rows, a_cols, a_vals, overflow = self.anomalies.fetch()
            if overflow:  # more anomalous points than the list holds: re-derive from the band
                a_rows, a_cols, a_vals = self._anomalies_from_band(verdict)
        else:
            a_rows, a_cols = np.nonzero(out["_anomaly"].numpy() & (out["verdict"] == 1).numpy()[:, None])
            a_vals = self.win.numpy()[a_rows, a_cols]
        self.timings["score_ms"] = (time.perf_counter() - t0) * 1e3
        t0 = time.perf_counter()
        self._bands = (host[2], host[3], verdict)
        written = self._verdicts(now, verdict, npts, a_rows, a_cols, a_vals)
        self.timings["verdict_ms"] = (time.perf_counter() - t0) * 1e3
        self.ticks += 1
        self.metrics.tick.observe(time.perf_counter() - t_tick)
        self.metrics.series_scored.inc(self.n_live)
        self.timings["tick_ms"] = (time.perf_counter() - t_tick) * 1e3
        return written

    def _anomalies_from_band(self, verdict):
        x = self.win.cpu().numpy()
        up, lo = self.out["upper"].cpu().numpy(), self.out["lower"].cpu().numpy()
        b = self.bound.cpu().numpy().astype(np.int64)[:, None]
        flag = (((b & 1) != 0) & (x > up)) | (((b & 2) != 0) & (x < lo))
        flag &= (verdict == 1)[:, None]
        rr, cc = np.nonzero(flag)
        return rr, cc, x[rr, cc]

    def _verdicts(self, now: float, verdict: np.ndarray, npts: np.ndarray, a_rows, a_cols, a_vals) -> Dict[str, str]:
        """Jobs with an anomalous metric (fail fast) and jobs past endTime finish;
        the others stay leased and untouched."""
        P, Wc = self.P, self.Wc
        bad_rows = np.nonzero(verdict == 1)[0]
        points: Dict[int, List[Tuple[float, float, str]]] = {}
        for rr, cc, vv in zip(np.asarray(a_rows).tolist(), np.asarray(a_cols).tolist(), np.asarray(a_vals).tolist()):
            plan_ref = self.row_plan[rr]
            if plan_ref is None:
                continue
            s = self.jobs[plan_ref[0]].series[plan_ref[1]]
            p, c = divmod(int(cc), Wc)
            points.setdefault(rr, []).append((s.cur_start + c * self.step, float(vv),
                                              s.cur_pods[p] if p < len(s.cur_pods) else ""))
        finish: Dict[str, Tuple[str, str, Optional[Dict]]] = {}
        for rr in bad_rows.tolist():
            plan_ref = self.row_plan[rr]
            if plan_ref is None or plan_ref[0] in finish:
                continue
            jid = plan_ref[0]
            p = self.jobs[jid]
            anomaly = {}
            for row, s in zip(p.rows, p.series):
                if verdict[row] != 1:
                    continue
                pts = sorted(points.get(row, []))
                vals: List[float] = []
                for ts, v, _ in pts:
                    vals += [ts, v]
                anomaly[s.alias] = {"tags": ",".join(sorted({t for _, _, t in pts if t})), "values": vals}
                self._last_anom[row] = pts[-1][0] if pts else now
            finish[jid] = (r.ST_COMPLETED_UNHEALTH, "anomaly detected in " + ",".join(sorted(anomaly)), anomaly)
        while self._ends and self._ends[0][0] <= now:
            _, jid = heapq.heappop(self._ends)
            p = self.jobs.get(jid)
            if p is None or jid in finish:
                continue
            seen = bool(npts[p.rows].sum() > 0)
            if seen and any(self.model_ok[row] for row in p.rows):
                finish[jid] = (r.ST_COMPLETED_HEALTH, "", None)
            elif seen:
                finish[jid] = (r.ST_COMPLETED_UNKNOWN, "missing historical data", None)
            else:
                finish[jid] = (r.ST_COMPLETED_UNKNOWN, "no current metric data", None)
        if not finish:
            return {}
        items = []
        for jid, (status, reason, anomaly) in finish.items():
            fields = {"status": status, "reason": reason, "claimed_by": "", "modified_ts": now,
                      "processingContent": f"scored by {self.worker_id} (resident engine)"}
            if anomaly:
                fields["anomalyInfo"] = json.dumps(anomaly)
            items.append((jid, fields))
        res = self.store.update_many(items, expect_claimed_by=self.worker_id)
        written = {}
        freed: List[int] = []  # every finished job's rows, released in ONE batch of device fills
        for (jid, fields), ok in zip(items, res):
            if ok:
                self.metrics.jobs.labels(status=fields["status"]).inc()
                written[jid] = fields["status"]
            p = self.jobs.pop(jid, None)
            if p is not None:
                up, lo, _ = self._bands
                for row, s in zip(p.rows, p.series):  # the finished job's last band stays exported
                    if row < len(up) and not math.isnan(up[row]):
                        self.metrics.export_band(s.hkey[1], s.hkey[2], s.hkey[3], float(up[row]), float(lo[row]),
                                                 self._last_anom.get(row))
                self.history.unwant([s.hkey for s in p.series], now)
                freed += p.rows
                self.slots.release(self._job_pods(p))
                self._app_ref(p, -1)
                for row in p.rows:
                    self._last_anom.pop(row, None)
        self._free_rows(freed)
        return written

    # ------------------------------------------------------------------ node integration
    def app_table(self) -> Tuple[List[Optional[Tuple[str, str]]], torch.Tensor]:
        """(app index -> name, None for a free index; ``[A, 2]`` device counters
        of the last tick: anomalous series, scored series)."""
        names = list(self._app_names)
        if not self.cap:
            return names, torch.zeros((len(names), 2), dtype=torch.int32, device=self.device)
        return names, self.app_stats[:len(names)]

    def _band_rows(self):
        up, lo, verdict = self._bands
        for jid, p in list(self.jobs.items()):
            for row, s in zip(p.rows, p.series):
                if row < len(up) and not math.isnan(up[row]):
                    yield (s.hkey[1], s.hkey[2], s.hkey[3], float(up[row]), float(lo[row]), self._last_anom.get(row))
