"""Continuous multi-metric jobs on the resident LSTM-autoencoder engine.

The reference brain scores a job with 3+ metrics with an LSTM model
(``docs/guides/design.md:84``; ``ML_ALGORITHM=lstm`` for 2+).  The per-job
path (:mod:`.multivariate`) trains one small model per job.  On a GPU node
the continuous LSTM jobs of every rank are served by ONE shared
LSTM-autoencoder per node, trained data-parallel across the ranks
(BASELINE configs 3 / 5 in the product, not only in the bench):

* entity = a continuous job; its metrics (sorted aliases, at most ``F``,
  absent ones zero-padded) are the features of one row of an
  :class:`~.lstm_engine.LstmShard`; the 7-day history of each metric comes
  from the node's resident keyed history (:mod:`.resident`: one query per
  metric family per tick, week-long loads only for new series) and is copied
  into the shard's per-feature rings when the job joins;
* every tick, on every rank in lockstep: the new minute of every entity is
  appended, ONE data-parallel Adam step runs on windows sampled from this
  rank's live entities (RC3: bucketed gradient all-reduce over RCCL, the
  rank's weight — 0 when it holds no LSTM job — and an "admitted entities"
  flag in the same collective), every rank's replica applies the same
  averaged step, so the replicas stay bit-identical; when any rank admitted
  entities, every rank joins a calibration pass (new rows' error levels,
  pooled spread); after a node re-formation the weights and Adam state are
  broadcast from rank 0 (RC4);
* the fused MFMA kernel scores every entity's newest window (bf16; fp8 e4m3
  with ``FOREMAST_LSTM_FP8=1``) → per-entity z-score against its calibrated
  error level → verdict; an anomalous entity finishes its job
  ``completed_unhealth`` naming every metric with its newest point, past
  ``endTime`` the job finishes ``completed_health``.
"""

from __future__ import annotations

import collections
import itertools
import json
import logging
import os
import time
from dataclasses import dataclass
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist

from ..parallel.roster import ChangeLog
from ..api import rest as r
from ..parallel import comm
from ..store.jobstore import JobStore
from ..utils.config import BrainConfig
from ..utils.metrics import BrainMetrics
from ..utils.timeutil import TimeFormatError, parse_rfc3339
from .lstm_engine import LstmShard
from .resident import Key, ResidentHistory
from .streaming import CALLER_SPLIT, is_continuous, series_of

log = logging.getLogger("foremast.lstm_monitor")

_ENC_STR = json.encoder.encode_basestring_ascii


def _jfloat(x: float) -> str:
    """``json.dumps`` of one float (repr; NaN / Infinity spelled as the json module does)."""
    if x != x:
        return "NaN"
    if x in (float("inf"), float("-inf")):
        return "Infinity" if x > 0 else "-Infinity"
    return repr(x)


def anomaly_info(t: float, pairs) -> str:
    """``json.dumps({alias: {"tags": "lstm", "values": [t, v]}, ...})`` for (alias, v) pairs,
    string-equal to it, without the encoder's per-call setup (~8 us a call: a tick on which
    500 jobs fail at once wrote 500 of these inside the detect latency)."""
    ts = _jfloat(float(t))
    return "{" + ", ".join(f'{_ENC_STR(a)}: {{"tags": "lstm", "values": [{ts}, {_jfloat(float(v))}]}}'
                           for a, v in pairs) + "}"


def lstm_features(doc, cfg: BrainConfig) -> Optional[List[Tuple[str, Key]]]:
    """(alias, series key) features of a continuous job the LSTM engine scores
    (``ML_ALGORITHM=lstm`` with 2+ metrics, ``auto`` with 3+), else None."""
    if not is_continuous(doc) or cfg.algorithm not in ("lstm", "auto"):
        return None
    feats = sorted(series_of(doc).items())
    if any(k[1].startswith(CALLER_SPLIT) or not k[3] for _, k in feats):
        return None
    need = 2 if cfg.algorithm == "lstm" else 3
    return feats if len(feats) >= need else None


@dataclass
class Entity:
    doc: Dict
    end_ts: float
    feats: List[Tuple[str, Key]]   # (alias, history key); the key may be None when ``hk`` is given
    row: int = -1
    external: bool = False   # a rollout job's joint model (brain/rollout.py): fed, verdicts read back
    hk: Optional[List[int]] = None          # history key hashes of the features
    app: Optional[Tuple[str, str]] = None   # (namespace, app)


class LstmMonitor:
    def __init__(self, store: JobStore, cfg: Optional[BrainConfig] = None, prom=None, device=None,
                 worker_id: str = "lstm-0", metrics: Optional[BrainMetrics] = None, step: float = 60.0,
                 clock=time.time, owns: Optional[Callable[[Dict], bool]] = None, ring_len: Optional[int] = None,
                 features: int = 5, window: Optional[int] = None, hidden: Optional[int] = None,
                 fp8: Optional[bool] = None, train_batch: int = 4096, min_capacity: int = 64, seed: int = 0,
                 history: Optional[ResidentHistory] = None, decode_threads: Optional[int] = None) -> None:
        from ..promql.client import PromClient
        self.store = store
        self.cfg = cfg or BrainConfig.from_env()
        self.prom = prom or PromClient()
        self.device = torch.device(device) if device is not None else (
            torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu"))
        self.gpu = self.device.type == "cuda"
        self.worker_id, self.step, self.clock, self.owns = worker_id, float(step), clock, owns
        self.metrics = metrics or BrainMetrics()
        self.F = int(features)
        R = ring_len or self.cfg.ring_len
        self.history = history or ResidentHistory(self.prom, self.device, R, self.step, clock=clock,
                                                  decode_threads=decode_threads)
        if fp8 is None:
            fp8 = os.environ.get("FOREMAST_LSTM_FP8", "0") not in ("0", "", "false")
        tb = train_batch if self.gpu else min(train_batch, 64)
        if self.gpu:  # the fused MFMA kernels are built for one hidden size
            from ..ops.lstm import H as KERNEL_H
            if (hidden or self.cfg.lstm_hidden) != KERNEL_H:
                log.warning("LSTM hidden size %s -> %d (the fused GPU kernels' size)", hidden or self.cfg.lstm_hidden,
                            KERNEL_H)
            hidden = KERNEL_H
        self.shard = LstmShard(max(1, min_capacity), R, self.F, window=window or self.cfg.lstm_window,
                               hidden=hidden or self.cfg.lstm_hidden, fp8=bool(fp8) and self.gpu,
                               device=self.device, threshold=self.cfg.lstm_threshold, train_batch=tb, seed=seed,
                               dtype=torch.bfloat16 if self.gpu else torch.float32, dp_overlap=False,
                               restat_every=1 << 30, season=self.cfg.season,
                               level_threshold=(self.cfg.lstm_level_threshold
                                                if self.cfg.lstm_level_threshold > 0 else None))
        for ring in self.shard.rings:
            ring.state.head, ring.state.length = 0, R
        self.shard.live = torch.zeros(0, dtype=torch.int64, device=self.device)
        self.jobs: Dict[str, Entity] = {}
        self.waiting: Dict[str, Entity] = {}
        self.row_job: List[Optional[str]] = [None] * self.shard.n
        self._used = np.zeros(self.shard.n, dtype=bool)   # row holds an entity (free / live lists in numpy)
        self.feat_rows = torch.full((self.shard.n, self.F), -1, dtype=torch.int64, device=self.device)
        self.padded = torch.zeros((self.shard.n, self.F), dtype=torch.bool, device=self.device)
        self.apps: Dict[Tuple[str, str], int] = {}
        self._app_names: List[Optional[Tuple[str, str]]] = [None]  # app 0: free rows (never reported)
        self.roster_log = ChangeLog()                               # (index, name) changes, drained by the node
        self.roster_version = 0
        self.t_cur = 0.0
        self.ticks = 0
        self.exchange_timeout = comm.exchange_timeout_s()
        # DP steps before the first calibration of a fresh node's model (FOREMAST_LSTM_PRETRAIN)
        # (800 on the GPU: a model calibrated after 200 steps keeps drifting under the per-tick
        # training, and its first ticks flag healthy series — profiles/lstm_detection_r3.md)
        self.pretrain_steps = int(os.environ.get("FOREMAST_LSTM_PRETRAIN", "800" if self.gpu else "20"))
        # the fresh model's initial training is spread over ticks (this many extra DP steps per
        # tick, every rank in lockstep) instead of stalling one lockstep tick for all of it;
        # entities admitted meanwhile are scored once it is done and they are calibrated
        self.pretrain_per_tick = int(os.environ.get("FOREMAST_LSTM_PRETRAIN_PER_TICK", "100" if self.gpu else "20"))
        self._uncalibrated: List[int] = []
        self._pending_cal = False   # some rank admitted entities while the model was pretraining
        self._pretraining = False
        self._calibrated = np.zeros(self.shard.n, dtype=bool)
        self._row_end = np.full(self.shard.n, np.inf)   # endTime per row (inf: free, external or open-ended)
        self._n_series = 0
        # the weights' CRC in the node table: every digest_every ticks and after a re-formation
        self.digest_every = int(os.environ.get("FOREMAST_LSTM_DIGEST_EVERY", "60"))
        self._digest: Optional[str] = None
        self._digest_tick = -1
        self.timings: Dict[str, float] = {}
        # external entities (rollout jobs' joint models): the newest value of each is fed by
        # the rollout engine (its canary pods' mean), and their verdicts are read back
        self.sync_history = True     # False: another monitor drives the shared history
        self._feed: Optional[Tuple[List[str], np.ndarray]] = None
        self._row_of: Dict[str, int] = {}   # admitted entity -> row (C-level lookups of a fed batch)
        self.hits: Dict[str, Tuple[float, np.ndarray]] = {}

    # ------------------------------------------------------------------ membership
    def is_mine(self, d) -> bool:
        return lstm_features(d, self.cfg) is not None and (self.owns is None or self.owns(d))

    def sync(self, steal_from=None) -> int:
        now = self.clock()
        docs = self.store.claim(self.worker_id, now=now, max_stuck_s=self.cfg.max_stuck_seconds, limit=10_000,
                                only=self.is_mine, steal_from=steal_from)
        for d in docs:
            if d["id"] in self.jobs or d["id"] in self.waiting:
                continue
            try:
                end_ts = parse_rfc3339(d.get("endTime", "")).timestamp()
            except TimeFormatError:
                end_ts = float("inf")
            feats = lstm_features(d, self.cfg)[:self.F]
            hk = [self.history.key_hash(k) for _, k in feats]
            self.waiting[d["id"]] = Entity(doc=d, end_ts=end_ts, feats=feats, hk=hk,
                                           app=(feats[0][1][2], feats[0][1][3]))
            self.history.want_h(hk, now, lambda i, feats=feats: feats[i][1])
        return len(docs)

    def release(self, pred: Callable[[Dict], bool]) -> int:
        now, back = self.clock(), []
        for jid, e in list(self.jobs.items()) + list(self.waiting.items()):
            if pred(e.doc):
                back.append((jid, {"status": r.ST_REPROGRESS, "claimed_by": "", "not_before": 0.0}))
                self._drop(jid, now)
        if back:
            self.store.update_many(back, expect_claimed_by=self.worker_id)
        return len(back)

    def attach(self, jid: str, feats: List[Tuple[str, Key]], end_ts: float, now: float) -> None:
        """Score a rollout job's metrics jointly (its first ``F`` aliases, sorted):
        the entity's rows hold the app's history, then the values :meth:`feed` gives."""
        feats = list(feats)[:self.F]
        self.attach_h(jid, [a for a, _ in feats], [self.history.key_hash(k) for _, k in feats],
                      (feats[0][1][2], feats[0][1][3]), end_ts, now, key_of=lambda i: feats[i][1])

    def attach_h(self, jid: str, aliases: Sequence[str], hk: Sequence[int], app: Tuple[str, str], end_ts: float,
                 now: float, key_of) -> None:
        """:meth:`attach` by history key hash (the rollout engine's plan columns carry
        them); ``key_of(i)``: the key tuple of feature i (asked only for keys without a
        history row yet)."""
        self.attach_many([(jid, aliases, hk, app, end_ts, key_of)], now)

    def attach_many(self, items, now: float) -> None:
        """:meth:`attach_h` of many jobs, ``items`` = (jid, aliases, hk, app, end_ts, key_of)
        tuples: one history reference call for all of them."""
        hks: List[int] = []
        owners: List[Tuple[int, int]] = []  # (item, feature) of each referenced key
        for t, (jid, aliases, hk, app, end_ts, _key_of) in enumerate(items):
            if jid in self.jobs or jid in self.waiting:
                continue
            n = min(self.F, len(hk))
            e = Entity(doc={"id": jid}, end_ts=end_ts, feats=[(a, None) for a in list(aliases)[:n]],
                       external=True, hk=list(hk)[:n], app=app)
            self.waiting[jid] = e
            hks += e.hk
            owners += [(t, f) for f in range(n)]
        if hks:
            self.history.want_h(hks, now, lambda i: items[owners[i][0]][5](owners[i][1]))

    def detach(self, jids, now: float) -> None:
        """Drop external entities (their rows freed in one batch of device fills)."""
        rows = []
        for jid in jids:
            self.hits.pop(jid, None)
            row = self._drop(jid, now, free_row=False)
            if row >= 0:
                rows.append(row)
        self._free_rows(rows)

    def feed(self, values: Dict[str, np.ndarray]) -> None:
        """Newest value of each external entity's features (NaN: keep the history's)."""
        jids = list(values)
        vals = np.full((len(jids), self.F), np.nan, dtype=np.float32)
        for i, j in enumerate(jids):
            v = np.asarray(values[j], dtype=np.float32)[:self.F]
            vals[i, :len(v)] = v
        self.feed_matrix(jids, vals)

    def feed_matrix(self, jids: Sequence[str], vals: np.ndarray) -> None:
        """:meth:`feed` as one ``[len(jids), F]`` float32 matrix (row i: job ``jids[i]``)."""
        self._feed = (jids, vals) if len(jids) else None

    def after_reform(self) -> None:
        """RC4: every rank adopts rank 0's weights and optimizer state after the
        node re-formed (a step may have been applied on some ranks only)."""
        if comm.active():
            # every weight and optimizer tensor in flight at once, each waited for with the
            # exchange deadline: a peer lost here raises CollectiveTimeout (the node re-forms)
            works = [(dist.broadcast(p.data, src=0, async_op=True), "weights")
                     for p in self.shard.model.parameters()]
            for st in self.shard.trainer.opt.state.values():
                for v in st.values():
                    if torch.is_tensor(v):
                        works.append((dist.broadcast(v.data if v.device == self.device else v, src=0,
                                                     async_op=True), "optimizer state"))
            for w, what in works:
                comm.wait_bounded(w, self.exchange_timeout, f"re-formation broadcast of the LSTM {what}")
            self.shard.packed = None
        self._digest = None

    def _drop(self, jid: str, now: float, free_row: bool = True, hks: Optional[list] = None) -> int:
        """Forget an entity; returns its row (-1: none), freed here unless ``free_row``
        is False (the caller frees a batch).  ``hks``: collect the history references to
        release instead of releasing them here (the caller releases a batch in one call)."""
        e = self.jobs.pop(jid, None) or self.waiting.pop(jid, None)
        if e is None:
            return -1
        self._row_of.pop(jid, None)
        if hks is None:
            self.history.unwant_h(e.hk, now)
        else:
            hks.extend(e.hk)
        if e.row < 0:
            return -1
        self._n_series -= len(e.feats)
        if free_row:
            self._free_rows([e.row])
        return e.row

    @property
    def n_live(self) -> int:
        return len(self.jobs)

    # ------------------------------------------------------------------ rows
    def _grow(self, cap: int) -> None:
        n = self.shard.n
        self.shard.grow(cap)
        self.row_job.extend([None] * (cap - n))
        self._used = np.concatenate([self._used, np.zeros(cap - n, dtype=bool)])
        fr = torch.full((cap, self.F), -1, dtype=torch.int64, device=self.device)
        fr[:n] = self.feat_rows
        pd = torch.zeros((cap, self.F), dtype=torch.bool, device=self.device)
        pd[:n] = self.padded
        self.feat_rows, self.padded = fr, pd
        self._calibrated = np.concatenate([self._calibrated, np.zeros(cap - n, dtype=bool)])
        self._row_end = np.concatenate([self._row_end, np.full(cap - n, np.inf)])

    def _free_rows(self, rows: List[int]) -> None:
        """Free rows in one batch: host bookkeeping, then one index fill per device array."""
        if not rows:
            return
        for row in rows:
            self.row_job[row] = None
        ra = np.asarray(rows, dtype=np.int64)
        self._used[ra] = False
        self._calibrated[ra] = False
        self._row_end[ra] = np.inf
        idx = torch.from_numpy(ra).to(self.device)
        self.feat_rows[idx] = -1
        self.padded[idx] = False
        self.shard.app_id[idx] = 0
        for ring in self.shard.rings:
            ring.data.index_fill_(0, idx, float("nan"))
        self._live_dirty = True

    def _app_index(self, app: Tuple[str, str]) -> int:
        i = self.apps.get(app)
        if i is None:
            i = self.apps[app] = len(self._app_names)
            self._app_names.append(app)
            self.roster_log.note(i, app)
            self.roster_version += 1
            if self.shard.app_stats.shape[0] < len(self._app_names):
                cap = self.shard.app_stats.shape[0]
                while cap < len(self._app_names):
                    cap *= 2
                self.shard.app_stats = torch.zeros((cap, 2), dtype=torch.int32, device=self.device)
        return i

    def _admit(self) -> List[int]:
        hist = self.history
        waiting = list(self.waiting.values())
        if not waiting:
            return []
        lens = np.fromiter((len(e.hk) for e in waiting), dtype=np.int64, count=len(waiting))
        allk = np.fromiter((h for e in waiting for h in e.hk), dtype=np.uint64, count=int(lens.sum()))
        ok = hist.ready_mask(allk)
        if ok.all():
            ready = waiting
        else:  # per entity: every feature's history ready
            cb = np.concatenate([[0], np.cumsum(~ok)])
            ends = np.cumsum(lens)
            ready = [e for e, nb in zip(waiting, (cb[ends] - cb[ends - lens]).tolist()) if nb == 0]
        if not ready:
            return []
        free = np.flatnonzero(~self._used)
        if len(free) < len(ready):
            cap = self.shard.n
            while cap - (self.shard.n - len(free)) < len(ready):
                cap *= 2
            self._grow(cap)
            free = np.flatnonzero(~self._used)
        free = free[:len(ready)].tolist()
        rows = free
        fr = np.full((len(ready), self.F), -1, dtype=np.int64)
        app_ids = np.empty(len(ready), dtype=np.int64)
        for i, (e, row) in enumerate(zip(ready, free)):
            del self.waiting[e.doc["id"]]
            self._row_of[e.doc["id"]] = row
            e.row = row
            self.jobs[e.doc["id"]] = e
            self.row_job[row] = e.doc["id"]
            self._n_series += len(e.hk)
            app_ids[i] = self._app_index(e.app)
        ra = np.asarray(rows, dtype=np.int64)
        self._used[ra] = True
        self._row_end[ra] = np.fromiter((np.inf if e.external else e.end_ts for e in ready), dtype=np.float64,
                                        count=len(ready))
        # feature rows of the resident history: one lookup for the whole batch
        flat = hist.rows_of_h([h for e in ready for h in e.hk])
        lens_r = np.fromiter((len(e.hk) for e in ready), dtype=np.int64, count=len(ready))
        ent = np.repeat(np.arange(len(ready)), lens_r)
        fi = np.arange(len(flat)) - np.repeat(np.cumsum(lens_r) - lens_r, lens_r)
        fr[ent, fi] = flat
        idx = torch.from_numpy(ra).to(self.device)
        self.shard.app_id[idx] = torch.from_numpy(app_ids).to(self.shard.app_id.device, self.shard.app_id.dtype)
        fr_t = torch.from_numpy(fr).to(self.device)
        self.feat_rows[idx] = fr_t
        self.padded[idx] = fr_t < 0
        # the week of each feature, from the resident ring (logical order, ending at t_last)
        ring = hist.ring
        cols = (torch.arange(hist.R, device=self.device) + ring.head) % hist.R
        vals = []
        for f in range(self.F):
            src = fr_t[:, f].clamp(min=0)
            v = ring.data.index_select(0, src).index_select(1, cols).float()
            vals.append(torch.where((fr_t[:, f] >= 0)[:, None], v, torch.zeros_like(v)))
        self.shard.write_rows(idx, vals)
        self._live_dirty = True
        return rows

    def _ingest(self) -> None:
        """Append the minutes the resident history gained since the last tick to
        every row (free rows get NaN, zero-padded features 0)."""
        hist = self.history
        if self.t_cur == 0.0:
            self.t_cur = hist.t_last
            return
        n_new = int(round((hist.t_last - self.t_cur) / self.step))
        if n_new <= 0:
            return
        R = hist.R
        for j in range(min(n_new, R)):
            age = min(n_new, R) - 1 - j                   # oldest new minute first
            col = (hist.ring.head + R - 1 - age) % R
            v = hist.ring.data[:, col].float()
            x = v[self.feat_rows.clamp(min=0)]
            if age == 0 and self._feed:  # external entities: the fed values of the newest minute
                x = self._fed(x)
            x = torch.where(self.padded, torch.zeros_like(x), x)
            x = torch.where((self.feat_rows >= 0) | self.padded, x, torch.full_like(x, float("nan")))
            self.shard.ingest_tick(x.contiguous())
        self.t_cur = hist.t_last

    def _fed(self, x: torch.Tensor) -> torch.Tensor:
        jids, vals = self._feed
        self._feed = None
        rows = np.fromiter(map(self._row_of.get, jids, itertools.repeat(-1)), dtype=np.int64, count=len(jids))
        ok = rows >= 0
        if not ok.any():
            return x
        idx = torch.from_numpy(rows[ok]).to(self.device)
        fv = torch.from_numpy(np.ascontiguousarray(vals[ok])).to(self.device)
        x = x.clone()
        x[idx] = torch.where(torch.isnan(fv), x[idx], fv)
        return x

    # ------------------------------------------------------------------ tick
    async def tick(self) -> Dict[str, str]:
        """One standalone tick: the scoring half, then the lockstep intake half (the
        entities admitted there are scored from the next tick on)."""
        written = await self.score_tick()
        await self.intake()
        return written

    async def intake(self) -> int:
        """The lockstep half (every rank runs it: the DP step and the calibration are
        collectives): week loads of new keys, admission, one training step (plus the
        initial training while it lasts), calibration of the admitted rows.  The next
        scoring half uses the model and the rows left here.  Returns the rows admitted."""
        t0 = time.perf_counter()
        now = self.clock()
        admitted: List[int] = []
        try:
            if self.sync_history:
                await self.history.load_pending(now)
            admitted = self._admit()
            if admitted:
                self.shard.refresh_stats()
        except Exception as e:  # noqa: BLE001 - the collectives below must still run on this rank
            log.exception("lstm data step failed: %s", e)
        if getattr(self, "_live_dirty", True):
            self.shard.live = torch.from_numpy(np.flatnonzero(self._used).astype(np.int64)).to(self.device)
            self._live_dirty = False
        has = int(self.shard.live.numel() > 0)
        flags = torch.full((1,), float(len(admitted)), dtype=torch.float32, device=self.device)
        self.shard.train_step(weight=float(has), flags=flags,
                              timeout_s=self.exchange_timeout if comm.active() else None)
        red = self.shard.trainer.last_flags
        self._uncalibrated += admitted
        # a fresh model's initial training, at most pretrain_per_tick extra steps per tick (the
        # step counts are equal on every rank: the trainers advance in lockstep)
        if red is not None and float(red[0]) > 0:
            self._pretraining = True  # the first entities anywhere start the initial training
        if self._pretraining and self.shard.trainer.steps < self.pretrain_steps:
            for _ in range(min(self.pretrain_per_tick, self.pretrain_steps - self.shard.trainer.steps)):
                self.shard.train_step(weight=float(has), timeout_s=self.exchange_timeout if comm.active() else None)
            self.timings["pretrain_steps"] = self.shard.trainer.steps
        pre_done = self.shard.trainer.steps >= self.pretrain_steps
        if pre_done and (self._pending_cal or (red is not None and float(red[0]) > 0)):
            # new rows (any rank) are calibrated together: a collective every rank joins
            self.shard.calibrate(min(self.shard.train_batch, 4096),
                                 rows=torch.tensor(self._uncalibrated, dtype=torch.long, device=self.device))
            self._calibrated[self._uncalibrated] = True
            self._uncalibrated = []
            self._pending_cal = False
        elif not pre_done and red is not None and float(red[0]) > 0:
            self._pending_cal = True
        self.timings["intake_ms"] = self.timings["train_ms"] = (time.perf_counter() - t0) * 1e3
        return len(admitted)

    async def score_tick(self) -> Dict[str, str]:
        """The scoring half: history advance, the newest minute into every row (fed
        values for external entities), scoring with the model of the last intake,
        verdicts; returns job -> status written."""
        t0 = time.perf_counter()
        now = self.clock()
        try:
            if self.sync_history:
                self.store.heartbeat(self.worker_id, now)
                await self.history.sync(now, load=False)
            self._ingest()
        except Exception as e:  # noqa: BLE001 - the lockstep intake half must still run on this rank
            log.exception("lstm ingest failed: %s", e)
        written: Dict[str, str] = {}
        self.hits = {}
        if not self.jobs:
            self.shard.app_stats.zero_()
            return written
        out = self.shard.score()
        v = out["verdict"].cpu().numpy()
        n = len(v)
        # only rows that flag or reach their endTime are visited (entities admitted while the
        # model was pretraining are scored once calibrated)
        cal = self._calibrated[:n]
        hit = (v == 1) & cal
        rows = np.nonzero(hit | (cal & (self._row_end[:n] <= now)))[0]
        newest = self._newest() if hit.any() else None
        items = []
        for row in rows.tolist():
            jid = self.row_job[row]
            e = self.jobs.get(jid) if jid is not None else None
            if e is None:
                continue
            if e.external:  # the rollout engine owns the job: it reads the verdict back
                if v[e.row] == 1:
                    self.hits[jid] = (self.history.t_last, newest[e.row])
                continue
            if v[e.row] == 1:
                nv = newest[e.row].tolist()
                aliases = [alias for alias, _k in e.feats]
                items.append((jid, {"status": r.ST_COMPLETED_UNHEALTH, "claimed_by": "", "modified_ts": now,
                                    "reason": "anomaly detected in " + ",".join(sorted(set(aliases))) + " (lstm)",
                                    "anomalyInfo": anomaly_info(self.history.t_last, dict(zip(aliases, nv)).items()),
                                    "processingContent": f"scored by {self.worker_id} (resident lstm)"}))
            elif now >= e.end_ts:
                items.append((jid, {"status": r.ST_COMPLETED_HEALTH, "claimed_by": "", "reason": "",
                                    "modified_ts": now,
                                    "processingContent": f"scored by {self.worker_id} (resident lstm)"}))
        if items:
            freed, hks = [], []
            for (jid, fields), ok in zip(items, self.store.update_many(items, expect_claimed_by=self.worker_id)):
                if ok:
                    written[jid] = fields["status"]
                row = self._drop(jid, now, free_row=False, hks=hks)
                if row >= 0:
                    freed.append(row)
            for st, n_st in collections.Counter(written.values()).items():
                self.metrics.jobs.labels(status=st).inc(n_st)
            self.history.unwant_h(hks, now)  # one bulk release (18 us a call per job before)
            self._free_rows(freed)
        self.ticks += 1
        self.metrics.series_scored.inc(self._n_series)
        self.timings["tick_ms"] = (time.perf_counter() - t0) * 1e3
        self.timings["verdicts_written"] = float(len(items))
        return written

    def _newest(self) -> np.ndarray:
        R = self.history.R
        col = (self.shard.rings[0].head + R - 1) % R
        return torch.stack([ring.data[:, col].float() for ring in self.shard.rings], 1).cpu().numpy()

    def model_digest(self) -> str:
        """CRC of the replica's weights (the node table shows every rank's: equal = in
        sync).  Recomputed every ``digest_every`` ticks and after a re-formation (it
        copies every weight to the host), the cached value otherwise."""
        if self._digest is not None and self.ticks - self._digest_tick < self.digest_every:
            return self._digest
        import zlib
        crc = 0
        for p in self.shard.model.parameters():
            crc = zlib.crc32(p.detach().float().cpu().numpy().tobytes(), crc)
        self._digest, self._digest_tick = f"{crc:08x}", self.ticks
        return self._digest

    def app_table(self):
        return list(self._app_names), self.app_counts()

    def roster_names(self):
        return self._app_names

    def app_counts(self) -> torch.Tensor:
        return self.shard.app_stats[:len(self._app_names)]
