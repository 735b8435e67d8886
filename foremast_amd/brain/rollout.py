"""One-shot canary / rollingUpdate jobs on the resident GPU engine.

The reference brain answers a rollout job by re-running the whole judgement
every cycle until ``endTime`` (``docs/guides/design.md:35,43``): fetch the
7-day history of each metric, the baseline pods' window (canary only) and the
new pods' window so far (``metricsquery.go:52-79``), fit the historical
model, run the pairwise test, lower the threshold if baseline and current
differ, detect.  :class:`RolloutMonitor` serves the same jobs from resident
state instead:

* admission (once per job, batched over every job claimed in a tick): job
  documents are decoded in one native batch (:mod:`.plans`) into columns; the
  history comes from the node's resident ring (:mod:`.resident`; fetched only
  for series the node has never held), the model is fitted ONCE on the
  history ending at the job's start — the reference job's historical window is
  fixed at creation, so refitting it every cycle would recompute the same
  model — and reduced to a forecast state per (job, metric) row: level,
  trend, the 16 forecast offsets of the current window's horizons, sigma,
  fitted grid point (h-step variance) and valid points.  The baseline pods'
  window ``[start - W, start]`` is fetched once, batched by pod family.  Rows,
  thresholds, pod slots and window maps are set with array operations over the
  admitted batch (no per-row Python objects);
* every tick: ONE range query per pod metric family for the newest minute of
  every pod of every running job → native keyed decode through ONE live pod
  index (``(namespace, pod)`` → slot; the tick block is ``[slot, family x
  minute]``, a family's body lands at its column offset) → one H2D → scatter
  kernel into each row's window at its own job-minute column → rank tests
  (MW-U / Wilcoxon / Kruskal, pods pooled) of baseline vs current → band /
  verdict / per-app counters / compacted anomaly list from the cached state
  (one launch, ``hw_detect_params_kernel``) → D2H;
* verdicts follow the reference state machine: an anomalous metric finishes
  the job ``completed_unhealth`` with its points and pod tags (fail fast);
  past ``endTime`` it finishes ``completed_health`` (current data seen) or
  ``completed_unknown``; in between the job stays leased — the engine renews
  all of its leases with one store heartbeat per tick instead of a write per
  job — and nothing is written;
* a tick is split in two (:meth:`score_tick`, then :meth:`intake`): verdicts
  of the running jobs first, then the claim and admission of new jobs — a new
  job's first current point is one step after its start (``metricsquery.go:52``),
  so admitting it after this tick's scoring delays nothing, and a deploy burst
  never delays the verdicts of the jobs already running;
* every per-tick host step is O(changed jobs): slots, the decode index, the
  window map and the app roster are updated in place for the admitted and
  finished jobs; band gauges are read from the last tick's host arrays at
  scrape time.

Multi-metric algorithms (``ML_ALGORITHM`` bivariate_normal / lstm / auto,
``docs/guides/design.md:53-89``) keep a moving_average_all row per metric and
add the job's joint model: the bivariate normal of its first two aliases (K8
fit at admission, Mahalanobis on the pod-mean windows every tick) or the LSTM
autoencoder over all of them (the node's resident LSTM engine,
:mod:`.lstm_monitor`, fed each tick with the canary pods' mean).

Jobs the resident engine cannot key (non-Prometheus sources, per-caller /
per-uri families, selectors that are not plain pod lists) stay with
:class:`~foremast_amd.brain.worker.BrainWorker` (:func:`is_rollout_keyable`).
"""

from __future__ import annotations

import collections
import heapq
import json
import logging
import os
import time
from typing import Callable, Dict, List, Optional, Tuple

import numpy as np
import torch

from ..api import rest as r
from ..ingest import native
from ..models import bivariate as biv_ref
from ..models import decompose as dec_ref
from ..models import detect as det_ref
from ..models import moving_average as ma_ref
from ..models import pairwise as pw_ref
from ..models import smoothing as sm_ref
from ..parallel.roster import ChangeLog
from ..store.jobstore import JobStore
from ..utils.config import BrainConfig
from ..utils.metrics import BrainMetrics
from . import plans as pl
from .plans import ALGORITHMS, STRATEGIES, PlanCols, RolloutPlan, RolloutSeries  # noqa: F401 (re-exported)
from .resident import Key, ResidentHistory, fetch_decode, quote_selector, range_url, range_url_quoted, re_alt

log = logging.getLogger("foremast.rollout")

HB = 16  # forecast offsets kept per row (kernels.HALF_HB): horizons 1..16 of the current window
_NO_ROWS = np.zeros(0, dtype=np.int64)
_NO_KEYS = np.zeros(0, dtype=np.uint64)


def plan_rollout(doc: Dict, cfg: BrainConfig, step: float = 60.0, window_cols: int = 11) -> Optional[RolloutPlan]:
    """The rollout-table plan of a job, or None when the resident engine cannot
    key it (memoised per job id, see :func:`plans.plan_many`)."""
    return pl.plan_rollout(doc, cfg.algorithm, step, window_cols)


def is_rollout_keyable(doc: Dict, cfg: BrainConfig) -> bool:
    return plan_rollout(doc, cfg) is not None


class PodSlots:
    """``(namespace, pod)`` key -> slot: a pod's row in the per-tick decode block
    (``[slot, family x minute]``: one slot serves every metric family).  Slots are
    reference counted by the jobs watching the pod (two jobs on one pod share it).
    Keys are the 64-bit pod keys of the job decoder; the map is the native decode
    index itself, updated in place when pods come and go (a released pod's key is
    retired, so a pod that keeps reporting after its job can never land in a
    reused slot), and looked up in batches (a dict stands in without the native
    library)."""

    def __init__(self, cap: int = 1024) -> None:
        self.cap = int(cap)
        self.refs = np.zeros(self.cap, dtype=np.int32)
        self.hash = np.zeros(self.cap, dtype=np.uint64)
        # next-fit allocation: new pods take the free slots at and after a cursor, in order.
        # Rollouts end roughly in the order they started, so the slots after the cursor are
        # the longest free and a tick's pods sit in slot order as its bodies list them: the
        # decode's writes to the tick block walk it forwards (a last-in-first-out free list
        # handed out slots in key-hash order, and the decode's random row writes cost ~3x)
        self.freemask = np.ones(self.cap, dtype=bool)
        self.cursor = 0
        self.grown = 0     # bumps when cap grows
        self.live = native.LiveKeyIndex("namespace", "pod") if native.available() else None
        self.index: Dict[int, int] = {}   # the map when the native library is missing
        self._n = 0

    def __len__(self) -> int:
        return self._n

    def slot_of(self, keys: np.ndarray) -> np.ndarray:
        """Slot of each key (-1: not held)."""
        u = np.ascontiguousarray(keys, dtype=np.uint64)
        if self.live is not None:
            return self.live.lookup(u)
        idx = self.index
        return np.fromiter((idx.get(h, -1) for h in u.tolist()), dtype=np.int64, count=len(u))

    def acquire(self, hashes: np.ndarray) -> np.ndarray:
        """One reference per occurrence of each key; returns the slot of each."""
        if not len(hashes):
            return np.zeros(0, dtype=np.int64)
        u, first, inv, cnt = np.unique(np.asarray(hashes, dtype=np.uint64), return_index=True, return_inverse=True,
                                       return_counts=True)
        slots = self.slot_of(u)
        new = np.nonzero(slots < 0)[0]
        # new keys in the order they were given (jobs in admission order, pods in row order:
        # the order the tick's bodies list them), so the native index's entries -- and its
        # next-element predictions -- are walked sequentially by the decode
        new = new[np.argsort(first[new], kind="stable")]
        if len(new):
            k = len(new)
            while self.cap - self._n < k:
                old = self.cap
                self.cap *= 2
                self.refs = np.concatenate([self.refs, np.zeros(old, dtype=np.int32)])
                self.hash = np.concatenate([self.hash, np.zeros(old, dtype=np.uint64)])
                self.freemask = np.concatenate([self.freemask, np.ones(old, dtype=bool)])
                self.cursor = old  # the fresh half is contiguous
                self.grown += 1
            c = self.cursor
            got = np.flatnonzero(self.freemask[c:])[:k] + c
            if len(got) < k:
                got = np.concatenate([got, np.flatnonzero(self.freemask[:c])[:k - len(got)]])
            self.freemask[got] = False
            self.cursor = int(got[-1]) + 1 if int(got[-1]) + 1 < self.cap else 0
            slots[new] = got
            self.hash[got] = u[new]
            if self.live is not None:
                self.live.set(u[new], got)
            else:
                self.index.update(zip(u[new].tolist(), got.tolist()))
            self._n += k
        np.add.at(self.refs, slots, cnt.astype(np.int32))
        return slots[inv]

    def release(self, hashes: np.ndarray) -> None:
        if not len(hashes):
            return
        u, cnt = np.unique(np.asarray(hashes, dtype=np.uint64), return_counts=True)
        slots = self.slot_of(u)
        ok = slots >= 0
        slots, cnt, u = slots[ok], cnt[ok], u[ok]
        np.subtract.at(self.refs, slots, cnt.astype(np.int32))
        gone = np.nonzero(self.refs[slots] <= 0)[0]
        if len(gone):
            gs = slots[gone]
            self.refs[gs] = 0
            if self.live is not None:
                self.live.retire(u[gone])
            else:
                for h in u[gone].tolist():
                    del self.index[h]
            self.freemask[gs] = True
            self._n -= len(gone)

    def table(self, fams: int):
        """The decode index (native): key -> slot."""
        return self.live


class RolloutMonitor:
    def __init__(self, store: JobStore, cfg: Optional[BrainConfig] = None, prom=None, device=None,
                 worker_id: str = "rollout-0", metrics: Optional[BrainMetrics] = None, step: float = 60.0,
                 window: int = 10, pods: int = 5, clock=time.time, owns: Optional[Callable[[Dict], bool]] = None,
                 history: Optional[ResidentHistory] = None, ring_len: Optional[int] = None,
                 min_capacity: int = 64, decode_threads: Optional[int] = None, apps_per_query: int = 256,
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
        self.decode_threads = max(1, int(decode_threads or native.default_threads()))
        self.apps_per_query = max(1, int(apps_per_query))
        self.claim_limit = claim_limit
        self.history = history or ResidentHistory(self.prom, self.device, ring_len or self.cfg.ring_len, self.step,
                                                  clock=clock, decode_threads=decode_threads,
                                                  apps_per_query=apps_per_query)
        self.min_capacity = max(1, int(min_capacity))
        self.jobs: Dict[str, RolloutPlan] = {}        # admitted (rows assigned)
        self.waiting: Dict[str, RolloutPlan] = {}     # claimed, history not resident yet
        self._ends: Dict[int, List[RolloutPlan]] = {}  # end minute -> admitted jobs ending in it
        self._end_keys: List[int] = []                 # heap of the minutes of _ends
        self._jplan: List[Optional[RolloutPlan]] = []  # job slot -> admitted plan (row_job indexes it)
        self._jfree: List[int] = []
        self.apps: Dict[Tuple[str, str], int] = {}
        self.roster_version = 0
        self.t_cur = 0.0                               # newest minute ingested into the windows
        self.ticks = 0
        self.tick_queries = 0
        self.admitted = 0
        self.cap = 0
        self._row_free = np.zeros(0, dtype=bool)       # free-row mask (admission takes the lowest)
        self._n_free = 0
        self.slots = PodSlots()
        self.fams: Dict[Tuple[str, str], int] = {}     # pod metric family -> index in the decode block
        self._fam_of_key: Dict[int, int] = {}          # family key (job decoder) -> index
        self._fam_rows = np.zeros(0, dtype=np.int64)   # live rows per family
        self._blocks: Dict[Tuple[int, int], List[torch.Tensor]] = {}
        self._block_i = 0
        self._srcmap_t: Optional[torch.Tensor] = None
        self._srcmap_geom = None                       # (slots cap, families, rows cap) it was built for
        self._srcmap_dirty: List[np.ndarray] = []      # rows changed since the device map was synced
        # cluster-affine ingest (parallel/affine.py): windows of another rank's clusters are
        # requested at admission and delivered by that rank in the tick's lockstep exchange
        self.router = None
        self._remote: List[Tuple[str, Tuple[str, str], float, int, List]] = []
        self.timings: Dict[str, float] = {}
        self._bands: Tuple[np.ndarray, np.ndarray, np.ndarray] = (np.zeros(0), np.zeros(0), np.zeros(0))
        # last bands of finished jobs' series, exported until their series come back: one entry
        # per retirement batch (plans, rows' plan index, series index, hash, upper, lower, last anomaly)
        self._done_chunks: "collections.deque" = collections.deque()
        self._done_n = 0
        self._ending: Dict[str, Tuple[str, str, Optional[Dict]]] = {}   # settled at scoring, written at intake
        self._end_ctx: Optional[Tuple[float, np.ndarray]] = None       # (scoring time, points seen) of the last scoring
        self._retire_pending: List[RolloutPlan] = []                   # fail-fast jobs written at scoring
        self.written_late: Dict[str, str] = {}                          # statuses the last intake wrote
        self._apps_dirty = False
        self._app_refs: Dict[Tuple[str, str], int] = {}
        self._app_names: List[Optional[Tuple[str, str]]] = []   # app index -> name (None: free index)
        self.roster_log = ChangeLog()                            # (index, name) changes, drained by the node
        self._app_free: List[int] = []
        self._app_new: List[Tuple[Tuple[str, str], List[int]]] = []
        self._app_gone: List[Tuple[str, str]] = []
        self._thr_cache: Dict[int, Tuple[float, int, float, int]] = {}   # (alias, metric) key -> threshold
        # window-corrected thresholds by (class, valid points): ONE table per distinct
        # (threshold, bound), built on the host in fp64 when a class first appears, read by
        # the detect kernel (no per-tick fp64 work on the device)
        self._thr_classes: Dict[Tuple[float, int], int] = {}
        self._lut: Optional[torch.Tensor] = None
        self._lut_n = self.P * self.Wc + 1
        # GPU scoring half: decoded block waiting for the device, tick scalars, record buffers,
        # captured HIP graphs of the scoring launches (FOREMAST_ROLLOUT_GRAPH=0: eager)
        self._pending: Optional[Tuple[torch.Tensor, int, int]] = None
        self._graphs: Dict[tuple, object] = {}
        self._src_devs: Dict[Tuple[int, int], torch.Tensor] = {}
        self.graph_on = os.environ.get("FOREMAST_ROLLOUT_GRAPH", "1") != "0"
        self.graph_replays = 0
        if self.gpu:
            self._tick_host = torch.zeros(4, dtype=torch.int32).pin_memory()
            self._tick_dev = torch.zeros(4, dtype=torch.int32, device=self.device)
        self._n_live = 0
        self._build_grid()
        self.anomalies = None
        self.metrics.add_band_source(f"rollout:{worker_id}", self._band_rows)
        # the joint LSTM autoencoder of 3+-metric jobs (ML_ALGORITHM lstm / auto): the node's
        # resident LSTM engine (brain/lstm_monitor.py) on this engine's history, data-parallel
        # across the ranks; every rank ticks it in lockstep
        self.joint_lstm = None
        self._lstm_rows: Dict[str, np.ndarray] = {}   # job -> its rows in feature (sorted alias) order
        # the LSTM jobs' rows as one [slots, F] matrix (a slot per job, -1: no row / free slot),
        # updated per attach / detach; its device copy is refreshed when it changed
        self._lstm_slot: Dict[str, int] = {}
        self._lstm_jids: List[Optional[str]] = []
        self._lstm_free: List[int] = []
        self._lstm_mat = np.zeros((0, 1), dtype=np.int64)
        self._lstm_cat = None   # device copy of the used part of _lstm_mat; None: stale
        if self.cfg.algorithm in ("lstm", "auto"):
            from .lstm_monitor import LstmMonitor
            self.joint_lstm = LstmMonitor(store, self.cfg, prom=self.prom, device=self.device,
                                          worker_id=worker_id + "-joint", metrics=self.metrics, step=step,
                                          clock=clock, history=self.history, ring_len=self.history.R,
                                          min_capacity=min_capacity,
                                          decode_threads=decode_threads)
            self.joint_lstm.sync_history = False

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
            "thr_cls": torch.zeros(cap, dtype=torch.int16, device=dev),
            # joint bivariate model of a 2-metric job, kept on its first alias's row
            "biv_mean": torch.zeros((cap, 2), **f32),
            "biv_cov": torch.zeros((cap, 3), **f32),
            "biv_ok": torch.zeros(cap, dtype=torch.bool, device=dev),
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
        grow = cap - n

        def ext(name, fill, dtype, shape=()):
            setattr(self, name, np.concatenate([getattr(self, name, np.zeros((0,) + shape, dtype)),
                                                np.full((grow,) + shape, fill, dtype=dtype)]))
        ext("model_ok", False, bool)
        ext("row_fam", -1, np.int64)
        ext("row_slot", -1, np.int64, (self.P,))
        ext("row_cs", 0.0, np.float64)      # cur_start of the row (anomaly timestamps)
        ext("row_s", -1, np.int64)          # series index in its PlanCols
        ext("row_job", -1, np.int64)        # job slot of the row (-1: free)
        ext("row_k", -1, np.int64)          # series index of the row within its job
        ext("last_anom", np.nan, np.float64)  # timestamp of the row's last anomalous point (band export)
        ext("biv_b", -1, np.int64)          # first-alias row of a bivariate job -> its second alias's row
        self._row_free = np.concatenate([self._row_free, np.ones(grow, dtype=bool)])
        self._n_free += grow
        self._srcmap_geom = None
        self.cap = cap
        if self.gpu:
            from ..ops import kernels as K
            # the scoring half's ONE copy back: [cap, 4] row records + the K9 list count
            self._rec_dev = torch.zeros(cap * 4 + 4, dtype=torch.float32, device=dev)
            self._rec_host = torch.zeros(cap * 4 + 4, dtype=torch.float32).pin_memory()
            self.anomalies = K.AnomalyBuffer(max(1024, 4 * cap), dev,
                                             count=self._rec_dev[cap * 4:cap * 4 + 1].view(torch.int32))
            self._graphs = {}

    def _free_rows(self, rows) -> None:
        ra = np.asarray(rows, dtype=np.int64)
        if not len(ra):
            return
        idx = torch.from_numpy(ra).to(self.device)
        self.win.index_fill_(0, idx, float("nan"))
        self.base.index_fill_(0, idx, float("nan"))
        self.app_id.index_fill_(0, idx, 0)
        self.row_job[ra] = -1
        self.row_k[ra] = -1
        self.biv_b[ra] = -1
        self.model_ok[ra] = False
        self._fam_count(self.row_fam[ra], -1)
        self.row_fam[ra] = -1
        self.row_slot[ra] = -1
        self.row_s[ra] = -1
        self._srcmap_dirty.append(ra)
        self._row_free[ra] = True
        self._n_free += len(ra)
        self._n_live -= len(ra)

    def _take_rows(self, n: int) -> np.ndarray:
        if self._n_free < n:
            used = self.cap - self._n_free
            cap = max(self.min_capacity, self.cap or 1)
            while cap < used + n:
                cap *= 2
            self._alloc(cap)
        out = np.flatnonzero(self._row_free)[:n]
        self._row_free[out] = False
        self._n_free -= len(out)
        return out.astype(np.int64)

    @property
    def n_live(self) -> int:
        return self._n_live

    def _take_jslots(self, n: int) -> np.ndarray:
        while len(self._jfree) < n:
            old = len(self._jplan)
            grow = max(64, old)
            self._jplan.extend([None] * grow)
            self._jfree = list(range(old + grow - 1, old - 1, -1)) + self._jfree
        out = self._jfree[len(self._jfree) - n:][::-1] if n else []
        del self._jfree[len(self._jfree) - n:]
        return np.asarray(out, dtype=np.int64)

    def _release_jslot(self, p: RolloutPlan) -> None:
        if p.jslot >= 0 and self._jplan[p.jslot] is p:
            self._jplan[p.jslot] = None
            self._jfree.append(p.jslot)
        p.jslot = -1

    def _end_push(self, p: RolloutPlan) -> None:
        """File an admitted job under the minute of its endTime (a job without a
        finite endTime never ends by time)."""
        if not np.isfinite(p.end_ts):
            return
        k = int(np.floor(p.end_ts / self.step))
        b = self._ends.get(k)
        if b is None:
            b = self._ends[k] = []
            heapq.heappush(self._end_keys, k)
        b.append(p)

    def _pop_ending(self, now: float, skip) -> List[RolloutPlan]:
        """Admitted jobs whose endTime has passed (not in ``skip``): whole minutes
        at once; the current minute's jobs one by one."""
        out: List[RolloutPlan] = []
        kn = int(np.floor(now / self.step))
        keys, jobs = self._end_keys, self.jobs
        while keys and keys[0] <= kn:
            k = keys[0]
            keep = []
            for p in self._ends[k]:
                if jobs.get(p.doc_id) is not p or p.doc_id in skip:
                    continue  # dropped / released, or finishing with an anomaly this tick
                (out if p.end_ts <= now else keep).append(p)
            if keep:
                self._ends[k] = keep
                break
            heapq.heappop(keys)
            del self._ends[k]
        return out

    # ------------------------------------------------------------------ membership
    def owns_affine(self, d) -> bool:
        """Cluster-affine mode: a job belongs to the rank that scrapes the cluster
        of its new pods (its history and current windows are then local)."""
        p = plan_rollout(d, self.cfg, self.step, self.Wc)
        return p is not None and self.router.local(p.first_fam[0])

    def _claimable(self, d) -> bool:
        return self._claimable_many([d])[0]

    def _claimable_many(self, docs) -> List[bool]:
        """Claim filter over a batch: one native decode for every unseen document."""
        plans = pl.plan_many(docs, self.cfg.algorithm, self.step, self.Wc)
        if self.owns is None:
            return [p is not None for p in plans]
        if self.router is not None and self.owns == self.owns_affine:
            return [p is not None and self.router.local(p.first_fam[0]) for p in plans]
        return [p is not None and self.owns(d) for p, d in zip(plans, docs)]

    def sync(self, steal_from=None) -> int:
        """Lease new keyable rollout jobs (that this rank owns)."""
        now = self.clock()
        t0 = time.perf_counter()
        docs = self.store.claim(self.worker_id, now=now, max_stuck_s=self.cfg.max_stuck_seconds,
                                limit=self.claim_limit, only_batch=self._claimable_many, steal_from=steal_from)
        t1 = time.perf_counter()
        plans = pl.plan_many(docs, self.cfg.algorithm, self.step, self.Wc)
        hist = self.history
        n = 0
        groups: Dict[int, Tuple[PlanCols, List[RolloutPlan]]] = {}
        for d, p in zip(docs, plans):
            if p is None or d["id"] in self.jobs or d["id"] in self.waiting:
                continue
            p.doc = d
            self.waiting[d["id"]] = p
            groups.setdefault(id(p.cols), (p.cols, []))[1].append(p)
            n += 1
        for c, ps in groups.values():  # history references: one call per decoded batch
            idx = np.concatenate([np.arange(p.s0, p.s0 + p.n) for p in ps])
            hist.want_h(c.u64[idx, 0].tolist(), now, lambda i, c=c, idx=idx: c.hkey_at(int(idx[i])))
        self.timings["claim_ms"] = (t1 - t0) * 1e3
        self.timings["plan_ms"] = (time.perf_counter() - t1) * 1e3
        self.timings["claimed"] = n
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
        self.history.unwant_h(p.cols.u64[p.s0:p.s0 + p.n, 0].tolist(), now)
        self._free_rows(p.rows)
        if len(p.rows):
            self._app_ref(p, -1)
            self.slots.release(p.pod_keys)
        self._release_jslot(p)
        if self._lstm_rows.pop(jid, None) is not None:
            self._lstm_unslot([jid])
            self.joint_lstm.detach([jid], now)
        p.rows = _NO_ROWS
        p.pod_keys = _NO_KEYS

    def _refresh_apps(self) -> None:
        """Apply the app-roster changes of the last admissions / verdicts.  App
        indices are stable (a freed index is reused by a later app), so a job
        finishing never renumbers the other rows; called at the end of the intake
        half and before scoring (a no-op then unless something changed since), so
        the roster :meth:`app_table` reports is the one the last tick's counters
        were accumulated under."""
        if not self._apps_dirty:
            return
        log = self.roster_log
        for a in self._app_gone:
            if self._app_refs.get(a, 0) <= 0 and a in self.apps:
                i = self.apps.pop(a)
                self._app_names[i] = None
                self._app_free.append(i)
                log.note(i, None)
        self._app_gone = []
        ids = np.empty(len(self._app_new), dtype=np.int32)
        apps, names, free = self.apps, self._app_names, self._app_free
        for k, (a, _rows) in enumerate(self._app_new):
            i = apps.get(a)
            if i is None:
                i = free.pop() if free else len(names)
                if i == len(names):
                    names.append(a)
                else:
                    names[i] = a
                apps[a] = i
                log.note(i, a)
            ids[k] = i
        if len(self._app_new):  # one device scatter for every admitted row
            lens = np.fromiter((len(rows) for _a, rows in self._app_new), dtype=np.int64, count=len(self._app_new))
            if lens.sum():
                rr = torch.from_numpy(np.concatenate([rows for _a, rows in self._app_new]).astype(np.int64))
                self.app_id[rr.to(self.device)] = torch.from_numpy(np.repeat(ids, lens)).to(self.device)
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
            self._app_new.append((p.app, p.rows))
        elif n <= 0:
            self._app_refs.pop(p.app, None)
            self._app_gone.append(p.app)
        self._apps_dirty = True

    # ------------------------------------------------------------------ admission
    async def _admit(self, now: float) -> int:
        hist = self.history
        waiting = list(self.waiting.values())
        if not waiting:
            return 0
        lens = np.fromiter((p.n for p in waiting), dtype=np.int64, count=len(waiting))
        ok = hist.ready_mask(np.concatenate([p.cols.u64[p.s0:p.s0 + p.n, 0] for p in waiting]))
        if not ok.all():  # per job: every one of its keys ready
            cb = np.concatenate([[0], np.cumsum(~ok)])
            ends = np.cumsum(lens)
            n_bad = cb[ends] - cb[ends - lens]
            ready = [p for p, nb in zip(waiting, n_bad.tolist()) if nb == 0]
        else:
            ready = waiting
        if not ready:
            return 0
        t0 = time.perf_counter()
        b = _Batch(ready, self.P)
        rows = self._take_rows(b.n)
        b.rows = rows
        starts = np.concatenate([[0], np.cumsum(b.lens)]).astype(np.int64)
        js = self._take_jslots(len(b.plans))
        for i, (p, j) in enumerate(zip(b.plans, js.tolist())):
            del self.waiting[p.doc_id]
            p.rows = rows[starts[i]:starts[i + 1]]
            p.jslot = j
            self._jplan[j] = p
            self.jobs[p.doc_id] = p
            self._end_push(p)
        self._n_live += b.n
        self.row_job[rows] = np.repeat(js, b.lens)
        self.row_k[rows] = np.arange(b.n) - np.repeat(starts[:-1], b.lens)
        self.row_s[rows] = b.s
        self.row_cs[rows] = b.f64[:, 0]
        t1 = time.perf_counter()
        self._set_row_params(b)
        self._assign_slots(b)
        t2 = time.perf_counter()
        self._fit(b)
        self._fit_joint(b)
        t3 = time.perf_counter()
        await self._load_windows(b)
        t4 = time.perf_counter()
        self.admitted += len(b.plans)
        for p in b.plans:
            self._app_ref(p, +1)
        self.timings.update(admit_ms=(time.perf_counter() - t0) * 1e3, admit_rows_ms=(t2 - t0) * 1e3,
                            admit_fit_ms=(t3 - t2) * 1e3, admit_windows_ms=(t4 - t3) * 1e3,
                            admitted=len(b.plans), admit_bookkeeping_ms=(t1 - t0) * 1e3)
        return len(b.plans)

    def _set_row_params(self, b: "_Batch") -> None:
        dev = self.device
        # thresholds per (alias, metric) class: one lookup per distinct class of the batch
        u, first, inv = np.unique(b.u64[:, 5], return_index=True, return_inverse=True)
        cache = self._thr_cache
        tab = np.empty((len(u), 4), dtype=np.float64)
        for k, (key, i) in enumerate(zip(u.tolist(), first.tolist())):
            t = cache.get(key)
            if t is None:
                c, s_ = b.cols_of(i), b.s_of(i)
                m = self.cfg.for_metric(c.alias[s_], c.hfam[s_][1])
                t = cache[key] = (m.threshold, m.bound, m.min_lower_bound, self._thr_class(m.threshold, m.bound))
            tab[k] = t
        thr = tab[inv]
        self.thr_cls[torch.from_numpy(b.rows).to(dev)] = torch.from_numpy(thr[:, 3].astype(np.int16)).to(dev)
        rows = torch.from_numpy(b.rows).to(dev)
        self.threshold[rows] = torch.from_numpy(thr[:, 0].astype(np.float32)).to(dev)
        self.bound[rows] = torch.from_numpy(thr[:, 1].astype(np.int8)).to(dev)
        self.min_lower[rows] = torch.from_numpy(thr[:, 2].astype(np.float32)).to(dev)
        self.start_min[rows] = torch.from_numpy(np.round(b.f64[:, 0] / self.step).astype(np.int32)).to(dev)
        self.win[rows] = float("nan")
        self.base[rows] = float("nan")

    def _thr_class(self, threshold: float, bound: int) -> int:
        """Class of (threshold, bound) in the device threshold table: row ``[cls, 0, n]``
        is the Sidak-corrected per-point level of a window of n valid points,
        ``[cls, 1, n]`` the lowered (pairwise) one (``models/detect.py``
        ``window_threshold``, computed in fp64 on the host once per class)."""
        key = (float(np.float32(threshold)), int(bound))
        k = self._thr_classes.get(key)
        if k is not None:
            return k
        k = self._thr_classes[key] = len(self._thr_classes)
        cfg, n = self.cfg, self._lut_n
        pts = torch.arange(n, dtype=torch.float64)
        thr = torch.full((n,), key[0], dtype=torch.float32)
        bnd = torch.full((n,), key[1], dtype=torch.int8)
        full, low = det_ref.effective_thresholds(thr, bnd, pts, cfg.pairwise_scale, cfg.window_correction)
        row = torch.stack([full, low]).float()
        if self._lut is None or self._lut.shape[0] <= k:
            cap = 8 if self._lut is None else 2 * self._lut.shape[0]
            lut = torch.zeros((cap, 2, n), dtype=torch.float32, device=self.device)
            if self._lut is not None:
                lut[:self._lut.shape[0]].copy_(self._lut)
            self._lut = lut
        self._lut[k].copy_(row.to(self.device))
        return k

    def _fit(self, b: "_Batch") -> None:
        """Fit every admitted row's model on its history ending at the job's
        start (grouped by how many of the ring's newest points that drops) and
        store the forecast state + per-column horizons."""
        hist = self.history
        drop = np.maximum(0, np.round((hist.t_last - b.f64[:, 2]) / self.step).astype(np.int64))
        hrows = hist.rows_of_h(b.u64[:, 0].tolist())
        Wc = self.Wc
        tiles = np.tile(np.arange(Wc), self.P)[None, :]
        for dv in np.unique(drop).tolist():
            sel = np.nonzero(drop == dv)[0]
            t_fit = hist.t_last - dv * self.step
            data, head, length = hist.gather(hrows[sel].tolist(), dv)
            st = self._fit_state(data, head, length)
            idx = torch.from_numpy(b.rows[sel]).to(self.device)
            for k, v in st.items():
                self.state[k][idx] = v.to(self.state[k].dtype)
            self.model_ok[b.rows[sel]] = (st["nvalid"] >= self.cfg.min_historical_points).cpu().numpy()
            off = np.round((b.f64[sel, 0] - t_fit) / self.step).astype(np.int64)
            hz = off[:, None] + tiles
            self.hz[idx] = torch.from_numpy(np.clip(hz, 1, 1 << 20).astype(np.int32)).to(self.device)

    def _fit_joint(self, b: "_Batch") -> None:
        """Joint models of the admitted multi-metric jobs (``ML_ALGORITHM`` bivariate_normal
        / auto): the bivariate normal of a job's first two aliases (sorted, as
        ``brain/worker.py`` pairs them), fitted on their 7-day histories ending at the
        job's start (K8 ``bivariate`` kernel on the GPU), kept on the first alias's row."""
        algo = self.cfg.algorithm
        if algo not in pl.JOINT_ALGORITHMS:
            return
        hist = self.history
        starts = np.concatenate([[0], np.cumsum(b.lens)]).astype(np.int64)
        ia, ib = [], []   # batch rows of each bivariate job's two aliases
        now = self.clock()
        attach = []       # the joint LSTM's new entities, referenced in one call
        for i, p in enumerate(b.plans):
            kind = pl.joint_kind(algo, p.n)
            if kind is None:
                continue
            al = [p.cols.alias[p.s0 + k] for k in range(p.n)]
            order = sorted(range(p.n), key=al.__getitem__)
            if kind == "lstm" and self.joint_lstm is not None:
                order = order[:self.joint_lstm.F]
                self._lstm_rows[p.doc_id] = p.rows[order]
                self._lstm_put(p.doc_id, p.rows[order])
                attach.append((p.doc_id, [al[k] for k in order], p.cols.u64[p.s0 + np.asarray(order), 0].tolist(),
                               p.app, p.end_ts, lambda i, p=p, order=order: p.cols.hkey_at(p.s0 + order[i])))
                continue
            ia.append(starts[i] + order[0])
            ib.append(starts[i] + order[1])
        if attach:
            self.joint_lstm.attach_many(attach, now)
        if not ia:
            return
        ia, ib = np.asarray(ia, dtype=np.int64), np.asarray(ib, dtype=np.int64)
        ha = hist.rows_of_h(b.u64[ia, 0].tolist())
        hb = hist.rows_of_h(b.u64[ib, 0].tolist())
        drop = np.maximum(0, np.round((hist.t_last - b.f64[ia, 2]) / self.step).astype(np.int64))
        dev = self.device
        for dv in np.unique(drop).tolist():
            sel = np.nonzero(drop == dv)[0]
            xa, head, length = hist.gather(ha[sel].tolist(), dv)
            xb, _, _ = hist.gather(hb[sel].tolist(), dv)
            k = len(sel)
            if self.gpu:
                from ..ops import kernels as K
                out = K.bivariate(xa, xb, head, length, torch.full((k, 1, 2), float("nan"), device=dev),
                                  torch.ones(k, device=dev), min_valid=self.cfg.min_historical_points)
                mean, cov = out["mean"], out["cov"]
                # jointly valid history points (the kernel's "count" is its count of anomalous current points)
                idx = (torch.arange(length, device=dev) + head) % xa.shape[1]
                count = (~(torch.isnan(xa.index_select(1, idx)) | torch.isnan(xb.index_select(1, idx)))).sum(1)
            else:
                idx = (torch.arange(length) + head) % xa.shape[1]
                fit = biv_ref.fit_bivariate(torch.stack([xa.index_select(1, idx), xb.index_select(1, idx)], 2))
                mean, cov, count = fit.mean, fit.cov, fit.count
            ra = torch.from_numpy(b.rows[ia[sel]]).to(dev)
            self.biv_mean[ra] = mean.float()
            self.biv_cov[ra] = cov.float()
            self.biv_ok[ra] = count.to(dev) >= self.cfg.min_historical_points
        self.biv_b[b.rows[ia]] = b.rows[ib]

    def _score_joint(self):
        """Bivariate jobs' points this tick: (first-alias rows, window columns, pod-mean
        values) where the squared Mahalanobis distance of the two aliases' pod-mean
        current values exceeds threshold^2 (``brain/batch.py`` ``score_bivariate``)."""
        rows = np.nonzero(self.biv_b >= 0)[0]
        if not len(rows):
            return None
        dev, P, Wc = self.device, self.P, self.Wc
        ra = torch.from_numpy(rows).to(dev)
        rb = torch.from_numpy(self.biv_b[rows]).to(dev)
        x = torch.nanmean(self.win[ra].view(-1, P, Wc), 1)
        y = torch.nanmean(self.win[rb].view(-1, P, Wc), 1)
        fit = biv_ref.BivariateFit(mean=self.biv_mean[ra], cov=self.biv_cov[ra], count=None)
        d2 = biv_ref.mahalanobis2(fit, torch.stack([x, y], 2))
        thr = self.threshold[ra]
        hit = (d2 > (thr * thr)[:, None]) & self.biv_ok[ra][:, None]
        i, c = torch.nonzero(hit, as_tuple=True)
        vals = x[i, c]
        i, c, vals = i.cpu().numpy(), c.cpu().numpy(), vals.cpu().numpy()
        return rows[i], c, vals

    def _algo_for(self, length: int) -> str:
        algo, m = self.cfg.algorithm, self.season
        if algo in pl.JOINT_ALGORITHMS:
            return "moving_average_all"   # the per-metric part; the joint model is _fit_joint's
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

    def _fam_index(self, fkeys: np.ndarray, cols_of, s_of) -> np.ndarray:
        """Family index of each row (by the decoder's family key; names interned once)."""
        out = np.empty(len(fkeys), dtype=np.int64)
        for i, k in enumerate(fkeys.tolist()):
            fi = self._fam_of_key.get(k)
            if fi is None:
                fam = cols_of(i).fam[s_of(i)]
                fi = self.fams.get(fam)
                if fi is None:
                    fi = self.fams[fam] = len(self.fams)
                self._fam_of_key[k] = fi
            out[i] = fi
        return out

    def _assign_slots(self, b: "_Batch") -> None:
        """Pod slots of the admitted rows: the first P current pods of each row; a
        job holds one reference per distinct pod (released when it finishes)."""
        P = self.P
        H, valid = b.cur_pod_keys()                           # [n, P] pod keys, mask
        jk = np.repeat(b.job, P)[valid.reshape(-1)]
        hk = H.reshape(-1)[valid.reshape(-1)]
        # distinct (job, pod): one reference each (sort by job then key, drop repeats)
        order = np.lexsort((hk, jk))
        jk, hk = jk[order], hk[order]
        keep = np.ones(len(hk), dtype=bool)
        keep[1:] = (jk[1:] != jk[:-1]) | (hk[1:] != hk[:-1])
        jk, hk_u = jk[keep], hk[keep]
        self.slots.acquire(hk_u)
        starts = np.searchsorted(jk, np.arange(len(b.plans) + 1))
        for i, p in enumerate(b.plans):
            p.pod_keys = hk_u[starts[i]:starts[i + 1]]
        # slot of every (row, pod): the keys are all live now
        u = np.unique(hk_u)
        us = self.slots.slot_of(u)
        pos = np.searchsorted(u, H.reshape(-1)).clip(0, max(len(u) - 1, 0))
        sl = np.where(valid.reshape(-1), us[pos] if len(u) else -1, -1).reshape(b.n, P)
        self.row_slot[b.rows] = sl
        fi = self._fam_index(b.u64[:, 1], b.cols_of, b.s_of)
        self.row_fam[b.rows] = fi
        self._fam_count(fi, +1)
        self._srcmap_dirty.append(b.rows)

    def _fam_count(self, fi: np.ndarray, sign: int) -> None:
        """Live rows per pod family (the tick queries only families with rows)."""
        fi = fi[fi >= 0]
        if not len(fi):
            return
        c = np.bincount(fi, minlength=len(self.fams))
        if len(self._fam_rows) < len(c):
            self._fam_rows = np.concatenate([self._fam_rows, np.zeros(len(c) - len(self._fam_rows), np.int64)])
        self._fam_rows[:len(c)] += sign * c

    def _srcmap(self) -> torch.Tensor:
        """Device ``[cap * P]`` src row of every (row, pod) in the tick block viewed as
        ``[slots * F, k]``: slot x F + family (-1: no pod).  Rebuilt when the slot
        capacity, the family count or the row capacity changes; otherwise only the
        rows admitted / freed since the last tick are written."""
        F = max(1, len(self.fams))
        geom = (self.slots.cap, F, self.cap)
        fam = self.row_fam[:, None]

        def rows_map(sel):
            s = self.row_slot[sel]
            f = fam[sel]
            return np.where((s >= 0) & (f >= 0), s * F + f, -1).astype(np.int32)
        if self._srcmap_t is None or self._srcmap_geom != geom:
            self._srcmap_t = torch.from_numpy(rows_map(slice(None)).reshape(-1)).to(self.device)
            self._srcmap_geom = geom
            self._srcmap_dirty = []
        elif self._srcmap_dirty:
            rows = np.unique(np.concatenate(self._srcmap_dirty))
            self._srcmap_dirty = []
            vals = torch.from_numpy(rows_map(rows)).to(self.device)
            self._srcmap_t.view(self.cap, self.P)[torch.from_numpy(rows).to(self.device)] = vals
        return self._srcmap_t

    async def _load_windows(self, b: "_Batch") -> None:
        """Baseline windows (fixed: ``[start - W, start]``) and any current points
        that already exist (a job claimed late), per (kind, window start, points):
        one query per pod family and group of jobs, every body of the group decoded
        through ONE key index over the group's pods (a family's body at its column
        offset), then gathered into the rows.  Rows are grouped with array ops."""
        t_last = self.history.t_last
        P, Wc = self.P, self.Wc
        specs = []  # (dst, batch rows, start per row, n per row, family key per row, pod column)
        hb = np.nonzero((b.i32[:, 6] > 0) & (b.i32[:, 5] > 0) & (b.i32[:, 1] > 0))[0]
        if len(hb):
            specs.append(("base", hb, b.f64[hb, 1], b.i32[hb, 1].astype(np.int64), b.u64[hb, 2], 4))
        cur_n = b.i32[:, 0].astype(np.int64)
        late = np.nonzero((cur_n > 0) & (b.f64[:, 0] <= t_last))[0]
        if len(late):
            n_late = np.minimum(cur_n[late], np.round((t_last - b.f64[late, 0]) / self.step).astype(np.int64) + 1)
            specs.append(("win", late, b.f64[late, 0], n_late, b.u64[late, 1], 2))
        for dst, idx, starts, ns_, fkeys, pc in specs:
            # group by (start, points); families within a group by their key
            gk = np.stack([starts.view(np.int64), ns_])
            _, ginv = np.unique(gk, axis=1, return_inverse=True)
            for g in range(int(ginv.max()) + 1 if len(ginv) else 0):
                sel = idx[ginv == g]
                start, n = float(starts[ginv == g][0]), int(ns_[ginv == g][0])
                await self._load_group(b, dst, sel, start, n, fkeys[ginv == g], pc)

    def _pods_strs(self, b: "_Batch", i: int, pc: int) -> Tuple[str, ...]:
        c, s = b.cols_of(i), b.s_of(i)
        return c.pods(int(c.i32[s, pc]), min(int(c.i32[s, pc + 1]), self.P))

    def _pod_matchers(self, b: "_Batch", chunk: np.ndarray, base: bool) -> str:
        """``{namespace=~"...",pod=~"..."}`` of the rows ``chunk`` (their jobs' pods)."""
        P = self.P
        nss, alts, loose = set(), set(), set()
        pk, ss = b._part_of[chunk], b.s[chunk]
        for k in np.unique(pk).tolist():
            cols = b.parts[k][0]
            for s_ in ss[pk == k].tolist():
                nss.add(cols.ns_at(s_))
                alt = cols.pods_alt(s_, base)
                if alt:                 # the job decoder's "a|b|c" of the row's pods
                    alts.add(alt)
                else:                   # rows of the Python parser
                    loose.update((cols.base_pods(s_) if base else cols.cur_pods(s_))[:P])
        pod_re = b"|".join(sorted(alts)).decode()
        if "." in pod_re:  # the one RE2 metacharacter a plain pod name can hold
            pod_re = pod_re.replace(".", "\\\\.")
        if loose:
            pod_re = "|".join(x for x in (pod_re, re_alt(loose)) if x)
        return f'{{namespace=~"{re_alt(nss)}",pod=~"{pod_re}"}}'

    async def _load_group(self, b: "_Batch", dst: str, sel: np.ndarray, start: float, n: int, fkeys: np.ndarray,
                          pc: int) -> None:
        P, Wc = self.P, self.Wc
        H, valid = b.pod_keys(pc, sel)                         # [k, P] keys of the rows' first P pods
        uk, inv = np.unique(H[valid], return_inverse=True)     # the group's distinct pods
        nl = len(uk)
        pos = np.full(H.shape, -1, dtype=np.int64)
        pos[valid] = inv
        ufk, fidx = np.unique(fkeys, return_inverse=True)      # families of the group
        fams = []
        for j in range(len(ufk)):
            i = int(sel[np.nonzero(fidx == j)[0][0]])
            c, s = b.cols_of(i), b.s_of(i)
            fams.append(c.base_fam[s] if dst == "base" else c.fam[s])
        if self.router is not None:  # windows of other ranks' clusters: requested, not fetched
            remote = np.array([not self.router.local(fams[j][0]) for j in range(len(fams))])
            if remote.any():
                for j in np.nonzero(remote)[0].tolist():
                    mj = fidx == j
                    rows_j = sel[mj]
                    # the request names the pods (the serving rank builds its query from them) ...
                    pods = list(dict.fromkeys((b.ns_of(int(i)), pod) for i in rows_j
                                              for pod in self._pods_strs(b, int(i), pc)))
                    # ... and the owner's scatter map is computed here once, from the rows' pod keys:
                    # (row, pod column) -> index of that pod in the request (-1: none)
                    ph = native.key_hashes([k[0] for k in pods], [k[1] for k in pods])
                    order = np.argsort(ph, kind="stable")
                    Hj, vj = H[mj], valid[mj]
                    at = np.searchsorted(ph[order], Hj).clip(0, max(len(pods) - 1, 0))
                    idx = np.where(vj & (ph[order][at] == Hj), order[at], -1) if len(pods) else \
                        np.full(Hj.shape, -1, dtype=np.int64)
                    self._remote.append((dst, fams[j], start, n, b.rows[rows_j].astype(np.int64), idx, pods))
                keep = ~remote[fidx]
                if not keep.any():
                    return
                return await self._load_group(b, dst, sel[keep], start, n, fkeys[keep], pc)
        F = len(fams)
        block_t = torch.full((max(nl, 1), F * Wc), float("nan"), dtype=torch.float32)
        if self.gpu:
            block_t = block_t.pin_memory()
        index = native.KeyTable.indexed(uk, np.arange(nl, dtype=np.int64), "namespace", "pod")
        reqs = []
        base = dst == "base"
        # a job's rows share its namespace and pods: the selector of a chunk of jobs is built and
        # URL-quoted once, and every family whose rows are the same jobs reuses it
        sel_of: Dict[bytes, str] = {}
        job = b.job[sel]
        for j, f in enumerate(fams):
            m_j = np.nonzero(fidx == j)[0]
            mine, jobs_j = sel[m_j], job[m_j]
            for g0 in range(0, len(mine), self.apps_per_query):
                chunk = mine[g0:g0 + self.apps_per_query]
                ck = jobs_j[g0:g0 + self.apps_per_query].tobytes()
                qsel = sel_of.get(ck)
                if qsel is None:
                    qsel = sel_of[ck] = quote_selector(self._pod_matchers(b, chunk, base))
                reqs.append((range_url_quoted(f[0], quote_selector(f[1]) + qsel, start, n, self.step), start, n,
                             j * Wc))
        ok = await fetch_decode(self.prom, reqs, [index] * len(reqs), block_t.numpy(), self.step,
                                self.decode_threads)
        if not all(ok):
            log.warning("%d of %d window queries failed (%s from %d)", ok.count(False), len(ok), dst, start)
        # gather: (group row, pod) -> block[pod, family]
        blk = block_t.to(self.device, non_blocking=True).view(max(nl, 1) * F, Wc)
        gi = torch.from_numpy(np.where(pos >= 0, pos * F + fidx[:, None], -1)).to(self.device)
        vals = blk[gi.clamp(min=0)]                            # [k, P, Wc]
        vals = torch.where((gi >= 0)[:, :, None], vals, torch.full_like(vals, float("nan")))
        rows = torch.from_numpy(b.rows[sel]).to(self.device)
        (self.base if dst == "base" else self.win).index_copy_(0, rows, vals.reshape(len(sel), P * Wc))

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
        """Cluster-affine lockstep exchange of this tick's remote window requests (the
        route changes of this tick's admissions; nothing when none was admitted).  The
        values arrive in one device buffer and are scattered into the rows' windows
        on the device through the scatter maps built at admission."""
        t0 = time.perf_counter()
        mine, self._remote = self._remote, []
        vals = await self.router.exchange([(f, st, n, pods) for _dst, f, st, n, _rows, _idx, pods in mine],
                                          self._serve_windows)
        P, Wc = self.P, self.Wc
        for (dst, f, st, n, rows, idx, pods), v in zip(mine, vals):
            ok = (rows >= 0) & (rows < self.cap)
            ok[ok] &= self.row_job[rows[ok]] >= 0      # rows retired since the request: skipped
            if not ok.any():
                continue
            rows_k, idx_k = rows[ok], idx[ok]
            gi = torch.from_numpy(idx_k).to(self.device)
            g = v[gi.clamp(min=0)]                                          # [k, P, n]
            g = torch.where((gi >= 0)[:, :, None], g, torch.full_like(g, float("nan")))
            block = torch.full((len(rows_k), P, Wc), float("nan"), dtype=torch.float32, device=self.device)
            m = min(n, Wc)
            block[:, :, :m] = g[:, :, :m]
            tgt = self.base if dst == "base" else self.win
            tgt.index_copy_(0, torch.from_numpy(rows_k).to(self.device), block.view(len(rows_k), P * Wc))
        self.timings["affine_ms"] = round((time.perf_counter() - t0) * 1e3, 3)
        self.timings["affine_bytes"] = float(self.router.last.get("bytes", 0))
        self.timings["affine_requests"] = float(self.router.last.get("requests", 0))

    def _tick_block(self, S: int, k: int, fill: bool = True):
        """Pinned decode block of the tick (NaN-filled unless ``fill`` is False: the
        decoder's threads fill it), one of two kept across ticks."""
        bufs = self._blocks.get((S, k))
        if bufs is None:
            bufs = [torch.empty((S, k), dtype=torch.float32) for _ in range(2)]
            if self.gpu:
                bufs = [b.pin_memory() for b in bufs]
            self._blocks = {(S, k): bufs}
        self._block_i ^= 1
        t = bufs[self._block_i]
        a = t.numpy()
        if fill:
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
        P = self.P
        F = max(1, len(self.fams))
        S = self.slots.cap
        t0 = time.perf_counter()
        srcmap = self._srcmap()
        fams = [(fam, fi) for fam, fi in self.fams.items() if fi < len(self._fam_rows) and self._fam_rows[fi] > 0]
        # the tick block is [slot, family x minute]: ONE pod index serves every family's body.
        # When the bodies cover every column the decoder's threads NaN-fill it in parallel
        native_fill = len({fi for _, fi in fams}) == F
        block_t, block = self._tick_block(S, F * k, fill=not native_fill)
        self.timings["ingest_prep_ms"] = (time.perf_counter() - t0) * 1e3
        self.timings["points"] = k
        index = self.slots.table(F)
        reqs = [(range_url(fam[0], fam[1], first, k, self.step), first, k, fi * k) for fam, fi in fams]
        self.tick_queries += len(reqs)
        t0 = time.perf_counter()
        ok = await fetch_decode(self.prom, reqs, [index] * len(reqs), block, self.step, self.decode_threads,
                                timings=self.timings, fill_nan=native_fill)
        self.timings["decode_ms"] = (time.perf_counter() - t0) * 1e3
        if not all(ok):
            return  # t_cur stays: the next tick fetches these minutes again
        src = block_t.view(S * F, k)
        if self.gpu:  # H2D + scatter are the first launches of the scoring half (_score_dev)
            self._pending = (src, int(round(first / self.step)), k)
        else:
            col0 = (int(round(first / self.step)) - self.start_min).to(torch.int32).contiguous()
            win = self.win.view(self.cap, P, self.Wc)
            sm = srcmap.view(self.cap, P).long()
            for j in range(k):
                c = (col0 + j).long()
                ok_r = ((c >= 0) & (c < self.Wc))[:, None] & (sm >= 0)
                vals = torch.where(ok_r, src[sm.clamp(min=0), j], torch.full(sm.shape, float("nan")))
                keep = ok_r & ~torch.isnan(vals)
                rr, pp = torch.nonzero(keep, as_tuple=True)
                win[rr, pp, c[rr]] = vals[rr, pp]
        self.t_cur = t_new

    # ------------------------------------------------------------------ GPU scoring half
    def _src_dev(self, rows: int, k: int) -> torch.Tensor:
        t = self._src_devs.get((rows, k))
        if t is None:
            t = torch.empty((rows, k), dtype=torch.float32, device=self.device)
            self._src_devs = {(rows, k): t}
        return t

    def _score_launch(self, pend) -> None:
        """Every device operation of the scoring half, stream-ordered and without a
        host synchronisation (captured once as a HIP graph and replayed): tick
        scalars H2D, tick block H2D, scatter into the windows (zeroing the per-app
        counters and the K9 count), rank tests, band / verdict / counters / K9 list
        / per-row record from the cached model state with the tabulated thresholds,
        record D2H.  Four copies and three kernels."""
        from ..ops import kernels as K
        cfg, P, Wc = self.cfg, self.P, self.Wc
        self._tick_dev.copy_(self._tick_host, non_blocking=True)
        zero = (self.app_stats.view(-1), self.anomalies.count)
        if pend is not None:
            src_host, _first, k = pend
            src = self._src_dev(src_host.shape[0], k)
            src.copy_(src_host, non_blocking=True)
            K.rollout_tick_scatter(self.win, P, Wc, src, self.start_min, self._tick_dev[0:1], self._srcmap_t, zero)
        else:
            K.rollout_tick_scatter(self.win[:0], P, Wc, self._src_dev(1, 1), self.start_min[:0], self._tick_dev[0:1],
                                   None, zero)
        pw_mode = pw_ref.PW_BY_NAME.get(cfg.pairwise_algorithm.upper(), pw_ref.PW_ALL)
        differs = None
        if pw_mode != pw_ref.PW_NONE:
            self.pw_out = K.rank_tests(self.base, self.win, pw_mode, cfg.pairwise_threshold, cfg.min_mann_white,
                                       cfg.min_wilcoxon, cfg.min_kruskal, want_pvals=False, out=self.pw_out,
                                       pods=(P, P), min_friedman=cfg.min_friedman)
            differs = self.pw_out["differs"]
        cap = self.cap
        spec = K.DetectSpec(horizons=self.hz, threshold=self.threshold, bound=self.bound, min_lower=self.min_lower,
                            cur=self.win, differs=differs, pw_scale=cfg.pairwise_scale,
                            min_valid=cfg.min_historical_points, want_band=True, app_id=self.app_id,
                            app_stats=self.app_stats, anomalies=self.anomalies,
                            pw_min_points=cfg.pairwise_min_points, shift_threshold=cfg.pairwise_shift,
                            shift_min_points=cfg.pairwise_shift_min_points, shift_one_step=cfg.pairwise_shift_one_step,
                            base_mean=self.pw_out["base_mean"] if differs is not None else None,
                            horizon_variance=cfg.horizon_variance, thr_lut=self._lut, thr_cls=self.thr_cls,
                            row_out=self._rec_dev[:cap * 4].view(cap, 4), start_min=self.start_min,
                            tick_min=self._tick_dev[1:2], last_ncol=Wc)
        st = dict(self.state)
        st.update(self.out)
        out = K.hw_detect_deferred(st, spec, self.m_detect, self.m_detect,
                                   grid=self.grid_all if cfg.horizon_variance else None)
        self.out = {k: out[k] for k in ("forecast", "upper", "lower", "count", "verdict", "score")}
        self._rec_host.copy_(self._rec_dev, non_blocking=True)

    def _score_dev(self):
        """The scoring half on the GPU: one graph replay (or the eager launches),
        one synchronisation, the host record; returns (verdict, points seen, upper,
        lower at the newest column, anomaly rows, columns, values)."""
        pend, self._pending = self._pending, None
        if self._lut is None:  # no class yet (rows admitted without _set_row_params): one neutral class
            self._thr_class(self.cfg.threshold, self.cfg.bound)
        th = self._tick_host.numpy()
        th[0] = pend[1] if pend is not None else 0
        th[1] = int(round(self.t_cur / self.step))
        self._srcmap()  # row map in sync with this tick's admissions / releases (in place)
        use_graph = self.graph_on and pend is not None and pend[2] == 1
        if use_graph:
            # every buffer the captured launches address that can be reallocated without a
            # capacity change (a replay would otherwise read a freed one)
            src_dev = self._src_dev(pend[0].shape[0], pend[2])
            key = (self.cap, tuple(pend[0].shape), pend[0].data_ptr(), src_dev.data_ptr(),
                   self._srcmap_t.data_ptr(), self._lut.data_ptr(), self.app_stats.data_ptr(),
                   self.win.data_ptr(), self.cfg.pairwise_algorithm)
            g = self._graphs.get(key)
            if g is None:
                self._score_launch(pend)          # this tick eagerly (allocates any outputs) ...
                torch.cuda.current_stream(self.device).synchronize()
                g = torch.cuda.CUDAGraph()        # ... and the next ones as one replay
                with torch.cuda.graph(g):
                    self._score_launch(pend)
                if len(self._graphs) >= 4:
                    self._graphs.clear()
                self._graphs[key] = g
            else:
                g.replay()
                self.graph_replays += 1
        else:
            self._score_launch(pend)
        torch.cuda.current_stream(self.device).synchronize()
        cap = self.cap
        rec = self._rec_host.numpy()
        rows = rec[:cap * 4].reshape(cap, 4)
        n_anom = int(rec[cap * 4:cap * 4 + 1].view(np.int32)[0])
        verdict = rows[:, 0].astype(np.int8)
        a_rows, a_cols, a_vals, overflow = self.anomalies.fetch(n_anom)
        if overflow:  # more anomalous points than the list holds: re-derive from the band
            a_rows, a_cols, a_vals = self._anomalies_from_band(verdict)
        return verdict, rows[:, 1], rows[:, 2].copy(), rows[:, 3].copy(), a_rows, a_cols, a_vals

    def _score(self) -> Dict[str, torch.Tensor]:
        """The scoring half on the CPU: the PyTorch reference models (fp64 Sidak
        thresholds per row, as the device table holds them)."""
        cfg = self.cfg
        valid = ~torch.isnan(self.win)
        npts = valid.sum(1)
        thr_f, thr_l = det_ref.effective_thresholds(self.threshold, self.bound, npts, cfg.pairwise_scale,
                                                    cfg.window_correction)
        pw_mode = pw_ref.PW_BY_NAME.get(cfg.pairwise_algorithm.upper(), pw_ref.PW_ALL)
        self.app_stats.zero_()
        differs = None
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
                           base_mean=torch.nanmean(self.base.float(), 1) if differs is not None else None,
                           shift_sigma=s["sigma"] if cfg.pairwise_shift_one_step else None)
        v = d.verdict.long()
        self.app_stats.index_put_((self.app_id.long(), torch.zeros_like(v)), (v == 1).int(), accumulate=True)
        self.app_stats.index_put_((self.app_id.long(), torch.ones_like(v)), (v >= 0).int(), accumulate=True)
        self.out = {"forecast": f, "upper": d.upper, "lower": d.lower, "count": d.count, "verdict": d.verdict,
                    "score": d.score, "_anomaly": d.anomaly, "npts": npts}
        return self.out

    # ------------------------------------------------------------------ ticks
    async def score_tick(self) -> Dict[str, str]:
        """The scoring half of a tick: heartbeat, window ingest, scoring, verdicts of
        the running jobs; returns job -> status written.  (The resident history is
        advanced in the intake half: scoring reads the admission-time model and the
        windows, not the week; admission needs the newest minute.)"""
        t_tick = time.perf_counter()
        now = self.clock()
        t_new = float(np.floor(now / self.step) * self.step)
        try:
            # inside the guard: a store error on this rank must not skip the lockstep
            # exchange of the intake half, or its peers' all_to_all would pair with another
            # collective
            self.store.heartbeat(self.worker_id, now)
        except Exception:  # noqa: BLE001
            if self.router is None:
                raise
            log.exception("rollout heartbeat failed (the affine exchange still runs)")
        self._refresh_apps()
        written: Dict[str, str] = {}
        if not self.jobs:
            self.t_cur = max(self.t_cur, t_new)
            self._bands = (np.zeros(0), np.zeros(0), np.zeros(0))
            if self.cap:
                self.app_stats.zero_()
            await self._tick_lstm(None)  # lockstep: the joint model's collectives run on every rank
            return written
        await self._ingest(t_new)
        t0 = time.perf_counter()
        last_c = None
        if self.gpu:
            verdict, npts, up, lo, a_rows, a_cols, a_vals = self._score_dev()
        else:
            out = self._score()
            last_c = ((int(round(self.t_cur / self.step)) - self.start_min).clamp(0, self.Wc - 1)).long()
            up = out["upper"].gather(1, last_c[:, None])[:, 0].numpy()
            lo = out["lower"].gather(1, last_c[:, None])[:, 0].numpy()
            verdict, npts = out["verdict"].numpy().astype(np.int8), out["npts"].float().numpy()
            a_rows, a_cols = np.nonzero(out["_anomaly"].numpy() & (out["verdict"] == 1).numpy()[:, None])
            a_vals = self.win.numpy()[a_rows, a_cols]
        self.timings["score_ms"] = (time.perf_counter() - t0) * 1e3
        t0 = time.perf_counter()
        joint = self._score_joint() if self.cfg.algorithm in pl.JOINT_ALGORITHMS else None
        if self.joint_lstm is not None and last_c is None:
            last_c = ((int(round(self.t_cur / self.step)) - self.start_min).clamp(0, self.Wc - 1)).long()
        lstm_hits = await self._tick_lstm(last_c)
        self._bands = (up, lo, verdict)
        written = self._verdicts(now, verdict, npts, a_rows, a_cols, a_vals, joint, lstm_hits)
        self.timings["verdict_ms"] = (time.perf_counter() - t0) * 1e3
        self.ticks += 1
        self.metrics.tick.observe(time.perf_counter() - t_tick)
        self.metrics.series_scored.inc(self.n_live)
        self.timings["tick_ms"] = (time.perf_counter() - t_tick) * 1e3
        return written

    async def intake(self) -> int:
        """The intake half of a tick: history of newly claimed jobs, admission, and
        (cluster-affine mode) the lockstep exchange of remote windows.  Returns the
        jobs admitted."""
        t0 = time.perf_counter()
        now = self.clock()
        n = 0
        self.written_late = {}
        try:
            self._settle_ending()
            self._retire_deferred()
            self.written_late = self._finish_ending()
            self.timings["ending_ms"] = (time.perf_counter() - t0) * 1e3
            t1 = time.perf_counter()
            await self.history.sync(now, load=False)  # the newest minute of every resident week
            self.timings["history_ms"] = (time.perf_counter() - t1) * 1e3
            await self.history.load_pending(now)
            n = await self._admit(now)
        except Exception:  # noqa: BLE001 - a store / Prometheus error: the lockstep parts below still run
            log.exception("rollout intake failed (retried next tick; the lockstep exchanges still run)")
        if self.router is not None:
            await self._route()  # every rank, every tick (collectives)
        if self.joint_lstm is not None:  # every rank, every tick: admission, DP step, calibration
            await self.joint_lstm.intake()
        # the roster changes of this tick's completions and admissions, applied here rather
        # than at the start of the next scoring half (the node table reported in between is
        # built before the intake half: the same roster either way)
        self._refresh_apps()
        self.timings["intake_ms"] = (time.perf_counter() - t0) * 1e3
        return n

    async def tick(self) -> Dict[str, str]:
        """One standalone tick: verdicts of the running jobs, then the admission of
        the jobs claimed by :meth:`sync`."""
        written = await self.score_tick()
        await self.intake()
        written.update(self.written_late)
        return written

    def _anomalies_from_band(self, verdict):
        x = self.win.cpu().numpy()
        up, lo = self.out["upper"].cpu().numpy(), self.out["lower"].cpu().numpy()
        b = self.bound.cpu().numpy().astype(np.int64)[:, None]
        flag = (((b & 1) != 0) & (x > up)) | (((b & 2) != 0) & (x < lo))
        flag &= (verdict == 1)[:, None]
        rr, cc = np.nonzero(flag)
        return rr, cc, x[rr, cc]

    def _lstm_put(self, jid: str, rows: np.ndarray) -> None:
        F = self.joint_lstm.F
        if self._lstm_mat.shape[1] != F:
            self._lstm_mat = np.full((max(64, len(self._lstm_mat)), F), -1, dtype=np.int64)
        if self._lstm_free:
            k = self._lstm_free.pop()
            self._lstm_jids[k] = jid
        else:
            k = len(self._lstm_jids)
            self._lstm_jids.append(jid)
            if k >= len(self._lstm_mat):
                self._lstm_mat = np.concatenate([self._lstm_mat, np.full_like(self._lstm_mat, -1)])
        self._lstm_slot[jid] = k
        self._lstm_mat[k] = -1
        self._lstm_mat[k, :min(F, len(rows))] = rows[:F]
        self._lstm_cat = None

    def _lstm_unslot(self, jids: Sequence[str]) -> None:
        ks = [self._lstm_slot.pop(j) for j in jids if j in self._lstm_slot]
        if ks:
            self._lstm_mat[ks] = -1
            for k in ks:
                self._lstm_jids[k] = None
            self._lstm_free.extend(ks)
            self._lstm_cat = None

    async def _tick_lstm(self, last_c: torch.Tensor) -> Dict[str, Tuple[float, np.ndarray]]:
        """The joint LSTM's tick (lockstep: every rank, every tick, jobs or not): feed
        each LSTM job's newest canary minute (pod mean per metric), one data-parallel
        step, score; returns job -> (time, values) of the jobs it flags."""
        if self.joint_lstm is None:
            return {}
        if self._lstm_rows:
            # [slots, F] rows of the jobs (one H2D per change of the job set); free slots and
            # missing features read NaN, and a free slot's job is None (not fed)
            n = len(self._lstm_jids)
            if self._lstm_cat is None:
                self._lstm_cat = torch.from_numpy(self._lstm_mat[:n].copy()).to(self.device)
            m = self._lstm_cat
            F = m.shape[1]
            ra = m.clamp(min=0).view(-1)
            col = last_c[ra]
            win = self.win[ra].view(len(ra), self.P, self.Wc)
            v = torch.nanmean(win.gather(2, col.view(-1, 1, 1).expand(-1, self.P, 1))[:, :, 0], 1)
            v = torch.where(m.view(-1) >= 0, v, torch.full_like(v, float("nan")))
            self.joint_lstm.feed_matrix(self._lstm_jids, v.view(n, F).float().cpu().numpy())
        else:
            self.joint_lstm.feed_matrix([], np.zeros((0, self.joint_lstm.F), dtype=np.float32))
        await self.joint_lstm.score_tick()  # the lockstep half runs in intake()
        return dict(self.joint_lstm.hits)

    def after_reform(self) -> None:
        if self.joint_lstm is not None:
            self.joint_lstm.after_reform()

    def model_digest(self) -> str:
        return self.joint_lstm.model_digest() if self.joint_lstm is not None else ""

    def _verdicts(self, now: float, verdict: np.ndarray, npts: np.ndarray, a_rows, a_cols, a_vals,
                  joint=None, lstm_hits=None) -> Dict[str, str]:
        """Jobs with an anomalous metric (fail fast) and jobs past endTime finish;
        the others stay leased and untouched.  ``joint``: (rows, columns, values) of the
        joint model's anomalous points; they flag the job and replace the anomalies of
        the first alias (``brain/worker.py`` ``_multivariate``)."""
        Wc = self.Wc
        bad_rows = np.nonzero(verdict == 1)[0]
        jpts: Dict[int, List[Tuple[float, float]]] = {}
        if joint is not None and len(joint[0]):
            for rr, cc, vv in zip(joint[0].tolist(), joint[1].tolist(), joint[2].tolist()):
                jpts.setdefault(rr, []).append((float(self.row_cs[rr]) + cc * self.step, float(vv)))
            bad_rows = np.union1d(bad_rows, np.fromiter(jpts, dtype=np.int64, count=len(jpts)))
        lstm_hits = {j: h for j, h in (lstm_hits or {}).items() if j in self.jobs}
        if lstm_hits:
            bad_rows = np.union1d(bad_rows, np.asarray([int(self.jobs[j].rows[0]) for j in lstm_hits], dtype=np.int64))
        row_job, jplan = self.row_job, self._jplan
        # anomalous points grouped by row in array form, each row's points ordered by
        # (time, value): its anomaly payload is one slice of an interleaved [t, v, ...] list
        ar = np.asarray(a_rows, dtype=np.int64)
        ac = np.asarray(a_cols, dtype=np.int64)
        av = np.asarray(a_vals, dtype=np.float64)
        keep = row_job[ar] >= 0 if len(ar) else np.zeros(0, dtype=bool)
        ar, ac, av = ar[keep], ac[keep], av[keep]
        pcs, cs = np.divmod(ac, Wc)
        ts = self.row_cs[ar] + cs * self.step
        order = np.lexsort((av, ts, ar))
        ar, ts, av, pcs = ar[order], ts[order], av[order], pcs[order]
        inter = np.empty(2 * len(ar), dtype=np.float64)
        inter[0::2], inter[1::2] = ts, av
        inter_l = inter.tolist()
        pcs_l = pcs.tolist()
        span: Dict[int, Tuple[int, int]] = {}
        if len(ar):
            st = np.flatnonzero(np.r_[True, ar[1:] != ar[:-1]])
            en = np.r_[st[1:], len(ar)]
            span = dict(zip(ar[st].tolist(), zip(st.tolist(), en.tolist())))
        finish: Dict[str, Tuple[str, str, Optional[Dict]]] = {}
        for rr in bad_rows.tolist():
            j = row_job[rr]
            if j < 0 or jplan[j].doc_id in finish:
                continue
            p = jplan[j]
            anomaly = {}
            hit = lstm_hits.get(p.doc_id)
            if hit is not None:  # the joint LSTM flags every metric at the scored minute (worker: _score_lstm)
                t_hit, vals_hit = hit
                al = [p.cols.alias[p.s0 + k] for k in range(p.n)]
                for f, k in enumerate(sorted(range(p.n), key=al.__getitem__)[:len(vals_hit)]):
                    anomaly[al[k]] = {"tags": "", "values": [float(t_hit), float(vals_hit[f])]}
                    self.last_anom[p.rows[k]] = float(t_hit)
                finish[p.doc_id] = (r.ST_COMPLETED_UNHEALTH, "anomaly detected in " + ",".join(sorted(anomaly)),
                                    anomaly)
                continue
            for k, row in enumerate(p.rows.tolist()):
                if row in jpts:  # the joint model's points replace this alias's own
                    jp = sorted(jpts[row])
                    anomaly[p.cols.alias[p.s0 + k]] = {"tags": "", "values": [x for tv in jp for x in tv]}
                    self.last_anom[row] = jp[-1][0]
                    continue
                if verdict[row] != 1:
                    continue
                sp = span.get(row)
                if sp is None:
                    anomaly[p.cols.alias[p.s0 + k]] = {"tags": "", "values": []}
                    self.last_anom[row] = now
                    continue
                lo_, hi_ = sp
                pods = p.cols.cur_pods(p.s0 + int(self.row_k[row]))
                names = {pods[q] for q in set(pcs_l[lo_:hi_]) if q < len(pods)}
                anomaly[p.cols.alias[p.s0 + k]] = {"tags": ",".join(sorted(n for n in names if n)),
                                                   "values": inter_l[2 * lo_:2 * hi_]}
                self.last_anom[row] = float(ts[hi_ - 1])
            finish[p.doc_id] = (r.ST_COMPLETED_UNHEALTH, "anomaly detected in " + ",".join(sorted(anomaly)), anomaly)
        # the jobs past endTime are settled in the intake half (after the node exchange):
        # nothing about them is news, and the fail-fast verdicts go out first
        self._end_ctx = (now, npts)
        return self._finish(finish, now, defer_retire=True)

    def _settle_ending(self) -> None:
        """Verdicts of the jobs whose endTime passed by the last scoring (points seen and
        model state of that scoring); written by :meth:`_finish_ending`."""
        ctx, self._end_ctx = self._end_ctx, None
        if ctx is None:
            return
        now, npts = ctx
        ending = self._pop_ending(now, ())  # this scoring's fail-fast jobs have left self.jobs
        if ending:  # past endTime: seen / model checks over every ending job's rows at once
            rr = np.concatenate([p.rows for p in ending])
            lens = np.fromiter((len(p.rows) for p in ending), dtype=np.int64, count=len(ending))
            starts = np.concatenate([[0], np.cumsum(lens)[:-1]])
            seen = np.add.reduceat((npts[rr] > 0).astype(np.int64), starts) > 0
            mok = np.add.reduceat(self.model_ok[rr].astype(np.int64), starts) > 0
            late: Dict[str, Tuple[str, str, Optional[Dict]]] = {}
            for p, sn, mk in zip(ending, seen.tolist(), mok.tolist()):
                if sn and mk:
                    late[p.doc_id] = (r.ST_COMPLETED_HEALTH, "", None)
                elif sn:
                    late[p.doc_id] = (r.ST_COMPLETED_UNKNOWN, "missing historical data", None)
                else:
                    late[p.doc_id] = (r.ST_COMPLETED_UNKNOWN, "no current metric data", None)
            self._ending.update(late)

    def _finish_ending(self) -> Dict[str, str]:
        """Write the settled endTime verdicts; they are forgotten only once written
        (a failing store write keeps them for the next intake, as it keeps the jobs)."""
        late = {j: v for j, v in self._ending.items() if j in self.jobs}
        if not late:
            self._ending = {}
            return {}
        written = self._finish(late, self.clock())
        self._ending = {}
        return written

    def _finish(self, finish: Dict[str, Tuple[str, str, Optional[Dict]]], now: float,
                defer_retire: bool = False) -> Dict[str, str]:
        """Write the final status of ``finish`` (job -> (status, reason, anomaly)) and
        retire the jobs (``defer_retire``: their rows, slots and history references are
        released at the next intake half, :meth:`_retire_deferred`)."""
        if not finish:
            return {}
        items = []
        content = f"scored by {self.worker_id} (resident engine)"
        for jid, (status, reason, anomaly) in finish.items():
            fields = {"status": status, "reason": reason, "claimed_by": "", "modified_ts": now,
                      "processingContent": content}
            if anomaly:
                fields["anomalyInfo"] = json.dumps(anomaly)
            items.append((jid, fields))
        res = self.store.update_many(items, expect_claimed_by=self.worker_id)
        written = {}
        counts: Dict[str, int] = {}
        done_plans: List[RolloutPlan] = []
        for (jid, fields), ok in zip(items, res):
            if ok:
                counts[fields["status"]] = counts.get(fields["status"], 0) + 1
                written[jid] = fields["status"]
            p = self.jobs.pop(jid, None)
            if p is not None:
                done_plans.append(p)
                self._app_ref(p, -1)
        for st, n in counts.items():
            self.metrics.jobs.labels(status=st).inc(n)
        if done_plans:
            if defer_retire:
                self._retire_pending.extend(done_plans)
            else:
                self._retire(done_plans, now)
        return written

    def _retire_deferred(self) -> None:
        plans, self._retire_pending = self._retire_pending, []
        if plans:
            self._retire(plans, self.clock())

    DONE_BANDS_MAX = 1 << 20   # rows of finished jobs whose last band stays exported

    def _retire(self, plans: List[RolloutPlan], now: float) -> None:
        """Release the finished jobs' rows, pod slots and history references in batches;
        their last bands stay exported (read at scrape time)."""
        up, lo, _ = self._bands
        freed = np.concatenate([p.rows for p in plans])
        lens = np.fromiter((len(p.rows) for p in plans), dtype=np.int64, count=len(plans))
        hk_all = np.concatenate([p.cols.u64[p.s0:p.s0 + p.n, 0] for p in plans])
        if len(up) >= self.cap and len(freed):
            u, l_ = up[freed], lo[freed]
            ok = ~np.isnan(u)
            if ok.any():
                pidx = np.repeat(np.arange(len(plans)), lens)[ok]
                k = self.row_k[freed][ok]
                s0 = np.fromiter((p.s0 for p in plans), dtype=np.int64, count=len(plans))
                srow = s0[pidx] + k
                hk = hk_all[ok]
                self._done_chunks.append((plans, pidx, srow, hk, u[ok], l_[ok], self.last_anom[freed][ok]))
                self._done_n += len(srow)
                while self._done_n > self.DONE_BANDS_MAX and len(self._done_chunks) > 1:
                    self._done_n -= len(self._done_chunks.popleft()[1])
        self.last_anom[freed] = np.nan
        self.history.unwant_h(hk_all.tolist(), now)
        self.slots.release(np.concatenate([p.pod_keys for p in plans]))
        self._free_rows(freed)
        for p in plans:
            self._release_jslot(p)
            # the plan object is memoised per job id (plans._PLANS): a later claim of the same
            # job must not find these rows and pod references, which may belong to others now
            p.rows = _NO_ROWS
            p.pod_keys = _NO_KEYS
        if self.joint_lstm is not None and self._lstm_rows:
            gone = [p.doc_id for p in plans if self._lstm_rows.pop(p.doc_id, None) is not None]
            if gone:
                self._lstm_unslot(gone)
                self.joint_lstm.detach(gone, now)

    # ------------------------------------------------------------------ node integration
    def app_table(self) -> Tuple[List[Optional[Tuple[str, str]]], torch.Tensor]:
        """(app index -> name, None for a free index; ``[A, 2]`` device counters
        of the last tick: anomalous series, scored series)."""
        return list(self._app_names), self.app_counts()

    def roster_names(self) -> List[Optional[Tuple[str, str]]]:
        return self._app_names

    def app_counts(self) -> torch.Tensor:
        n = len(self._app_names)
        if not self.cap:
            return torch.zeros((n, 2), dtype=torch.int32, device=self.device)
        return self.app_stats[:n]

    def _band_rows(self):
        up, lo, verdict = self._bands
        seen = set()
        la = self.last_anom
        for jid, p in list(self.jobs.items()):
            hk = p.cols.u64[p.s0:p.s0 + p.n, 0].tolist()
            for k, row in enumerate(p.rows.tolist()):
                if row < len(up) and up[row] == up[row]:
                    seen.add(hk[k])
                    key = p.cols.hkey_at(p.s0 + k)
                    an = float(la[row])
                    yield (key[1], key[2], key[3], float(up[row]), float(lo[row]), an if an == an else None)
        # finished jobs: the newest band of each series that is not live again
        for plans, pidx, srow, hk, u, l_, an in reversed(list(self._done_chunks)):
            for i, s, h, uu, ll, aa in zip(pidx.tolist(), srow.tolist(), hk.tolist(), u.tolist(), l_.tolist(),
                                           an.tolist()):
                if h in seen:
                    continue
                seen.add(h)
                key = plans[i].cols.hkey_at(s)
                yield (key[1], key[2], key[3], uu, ll, aa if aa == aa else None)


class _Batch:
    """The rows of one admission batch, gathered from the plans' columns (grouped
    by the PlanCols they came from)."""

    def __init__(self, plans: List[RolloutPlan], P: int) -> None:
        groups: Dict[int, Tuple[PlanCols, List[RolloutPlan]]] = {}
        for p in plans:
            groups.setdefault(id(p.cols), (p.cols, []))[1].append(p)
        self.plans: List[RolloutPlan] = []
        self.parts: List[Tuple[PlanCols, int, int]] = []   # (cols, first batch row, end)
        sidx, f64, i32, u64 = [], [], [], []
        n = 0
        for cols, ps in groups.values():
            s0 = np.fromiter((p.s0 for p in ps), dtype=np.int64, count=len(ps))
            ln = np.fromiter((p.n for p in ps), dtype=np.int64, count=len(ps))
            tot = int(ln.sum())
            s = np.repeat(s0 - (np.cumsum(ln) - ln), ln) + np.arange(tot)
            sidx.append(s)
            f64.append(cols.f64[s])
            i32.append(cols.i32[s])
            u64.append(cols.u64[s])
            self.parts.append((cols, n, n + tot))
            self.plans += ps
            n += tot
        self.n = n
        self.P = P
        self.s = np.concatenate(sidx) if sidx else np.zeros(0, np.int64)
        self.f64 = np.concatenate(f64) if f64 else np.zeros((0, 3))
        self.i32 = np.concatenate(i32) if i32 else np.zeros((0, 7), np.int32)
        self.u64 = np.concatenate(u64) if u64 else np.zeros((0, 6), np.uint64)
        self.lens = np.fromiter((p.n for p in self.plans), dtype=np.int64, count=len(self.plans))
        self.job = np.repeat(np.arange(len(self.plans)), self.lens)   # batch row -> plan index
        self._part_of = np.concatenate([np.full(hi - lo, k, dtype=np.int64) for k, (_, lo, hi) in
                                        enumerate(self.parts)]) if self.parts else np.zeros(0, np.int64)
        self.rows = np.zeros(0, np.int64)

    def cols_of(self, i: int) -> PlanCols:
        return self.parts[int(self._part_of[i])][0]

    def s_of(self, i: int) -> int:
        return int(self.s[i])

    def ns_of(self, i: int) -> str:
        return self.cols_of(i).ns_at(self.s_of(i))

    def alias_metric(self):
        for cols, lo, hi in self.parts:
            for s in self.s[lo:hi].tolist():
                yield cols.alias[s], cols.hfam[s][1]

    def pod_keys(self, pc: int = 2, sel: Optional[np.ndarray] = None) -> Tuple[np.ndarray, np.ndarray]:
        """``[n, P]`` keys of each row's first P pods (``pc`` 2: current, 4: baseline)
        and the valid mask; ``sel``: only these batch rows."""
        P = self.P
        sel = np.arange(self.n) if sel is None else np.asarray(sel, dtype=np.int64)
        H = np.zeros((len(sel), P), dtype=np.uint64)
        valid = np.zeros((len(sel), P), dtype=bool)
        K = np.arange(P)[None, :]
        part = self._part_of[sel]
        for k, (cols, _lo, _hi) in enumerate(self.parts):
            m = np.nonzero(part == k)[0]
            if not len(m):
                continue
            rows = sel[m]
            q0 = self.i32[rows, pc].astype(np.int64)[:, None]
            nq = np.minimum(self.i32[rows, pc + 1], P)[:, None]
            v = K < nq
            idx = np.where(v, q0 + K, 0)
            H[m] = np.where(v, cols.pod_u64[idx] if len(cols.pod_u64) else 0, 0)
            valid[m] = v
        return H, valid

    def cur_pod_keys(self) -> Tuple[np.ndarray, np.ndarray]:
        return self.pod_keys(2)

    def pod_key_bytes(self, i: int, pc: int) -> bytes:
        """Identity of a row's first P pods (its pod keys), for caching their names."""
        c, s = self.cols_of(i), self.s_of(i)
        q0, nq = int(c.i32[s, pc]), min(int(c.i32[s, pc + 1]), self.P)
        return c.pod_u64[q0:q0 + nq].tobytes()
