"""GPU-resident streaming scoring engine for one shard of series.

One ``StreamingShard`` per rank (one process per GPU).  It owns:

* the history ring ``[N, R]`` (bf16) and the current/baseline windows
  ``[N, P*W]`` in HBM;
* per-series config (threshold / bound / min_lower_bound, app id);
* preallocated outputs, so a scoring tick allocates nothing and can be
  captured into a HIP graph.

A tick is:  ``ingest_tick`` (K10: new per-pod points in, oldest graduate to
history)  →  ``score``: pairwise rank tests (K5/K11) → model fit + forecast +
band + verdict in ONE launch (K2/K3 + fused K9) → per-app health counts
(atomics in the same launch).  Cross-rank aggregation is
:mod:`foremast_amd.parallel.health`.

On CPU (tests, no GPU) the same API runs the PyTorch reference scorers.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, Optional, Tuple

import numpy as np
import torch

from ..ingest.ringbuffer import HistoryRing, WindowRing
from ..models import detect as det_ref
from ..models import moving_average as ma_ref
from ..models import pairwise as pw_ref
from ..models import smoothing as sm_ref
from ..utils.config import BrainConfig

OVERLAP_MIN_SERIES = 16384  # StreamingShard.overlap_pairwise default threshold

ALGO_MODE = {"exponential_smoothing": sm_ref.MODE_ES, "double_exponential_smoothing": sm_ref.MODE_DES,
             "holt_winters": sm_ref.MODE_HW}


@dataclass
class ShardSpec:
    n_series: int
    ring_len: int = 10080
    season: int = 1440
    pods: int = 5
    window: int = 10
    algorithm: str = "holt_winters"
    pairwise: str = "ALL"
    dtype: torch.dtype = torch.bfloat16
    n_apps: int = 1
    want_band: bool = True
    # Holt-Winters model cache: refit (64-point grid over the whole window) every
    # ``refit_every`` ticks; in between the fitted state is advanced by the graduated
    # point and the window scored from it in O(1) per series (1 = refit every tick)
    refit_every: int = 1
    extra: Dict = field(default_factory=dict)


class StreamingShard:
    def __init__(self, spec: ShardSpec, cfg: Optional[BrainConfig] = None, device="cpu",
                 app_id: Optional[torch.Tensor] = None, threshold: Optional[torch.Tensor] = None,
                 bound: Optional[torch.Tensor] = None, min_lower: Optional[torch.Tensor] = None,
                 app_stats: Optional[torch.Tensor] = None, verdict_out: Optional[torch.Tensor] = None) -> None:
        """``app_stats`` / ``verdict_out``: optional caller-owned outputs (e.g. the
        fused health record of :class:`HealthAggregator`) the tick writes in place."""
        self.spec = spec
        self.cfg = cfg or BrainConfig()
        self.device = torch.device(device)
        self.gpu = self.device.type == "cuda"
        N, P, W = spec.n_series, spec.pods, spec.window
        self.hist = HistoryRing(N, spec.ring_len, spec.dtype, self.device)
        self.cur = WindowRing(N, P, W, self.device)
        self.base = torch.full((N, P * W), float("nan"), dtype=torch.float32, device=self.device)
        kw = dict(device=self.device)
        self.threshold = (threshold if threshold is not None
                          else torch.full((N,), self.cfg.threshold, dtype=torch.float32, **kw))
        self.bound = bound if bound is not None else torch.full((N,), self.cfg.bound, dtype=torch.int8, **kw)
        self.min_lower = (min_lower if min_lower is not None
                          else torch.full((N,), self.cfg.min_lower_bound, dtype=torch.float32, **kw))
        self.app_id = app_id if app_id is not None else torch.zeros(N, dtype=torch.int32, **kw)
        self.refresh_thresholds()
        if app_stats is not None:
            if app_stats.dtype != torch.int32 or app_stats.dim() != 2 or app_stats.shape[1] != 2 \
                    or not app_stats.is_contiguous() or app_stats.device != self.device:
                raise ValueError("app_stats must be contiguous int32 [A, 2] on the shard's device")
            self.app_stats = app_stats
        else:
            self.app_stats = torch.zeros((max(spec.n_apps, 1), 2), dtype=torch.int32, **kw)
        if N and app_id is not None:
            lo, hi = int(self.app_id.min()), int(self.app_id.max())  # one-time sync at setup
            if lo < 0 or hi >= self.app_stats.shape[0]:
                raise ValueError(f"app_id range [{lo}, {hi}] outside the app table of {self.app_stats.shape[0]}")
        self.algorithm = spec.algorithm
        self.mode = ALGO_MODE.get(spec.algorithm)
        self.pw_mode = pw_ref.PW_BY_NAME.get(spec.pairwise.upper(), pw_ref.PW_ALL)
        g = sm_ref.make_grid(self.mode if self.mode is not None else sm_ref.MODE_HW,
                             self.cfg.hw_alpha, self.cfg.hw_beta, self.cfg.hw_gamma)
        self.grid = g.to(self.device)
        C = P * W
        self.horizons = torch.tensor(self.cur.horizons(), dtype=torch.int32, device=self.device)
        self._h_slots = None  # pinned horizon rows per window slot (see _refresh_horizons)
        self._h_dev = None    # the same rows on the device: eager ticks point at a row, no copy
        self._h_buf = self.horizons
        self._stats_zeroed = False
        self.out: Dict[str, torch.Tensor] = {}
        self._verdict_out = verdict_out
        if verdict_out is not None:
            if verdict_out.dtype != torch.int8 or verdict_out.shape != (N,) or verdict_out.device != self.device:
                raise ValueError(f"verdict_out must be int8 [{N}] on the shard's device")
            self.out["verdict"] = verdict_out
        self.pw_out: Dict[str, torch.Tensor] = {}
        # K9: compacted anomalous points of the current window (GPU), enabled via enable_anomaly_list()
        self.anomalies = None
        # HIP-graph tick (tick_graph): per-tick ring state lives in device memory
        self._graph = None
        self._graph_io = None
        self._graphs: Dict[tuple, tuple] = {}   # io buffers -> (graph, post captured, outputs)
        self._side = None                # side HIP stream for the rank tests (overlap_pairwise)
        # rank tests on a side stream beside the fit (deferred detection) from OVERLAP_MIN_SERIES
        # series; below, before the fit on the main stream with the detection fused into the
        # fit (the side stream's join and the separate detection kernel cost more than the
        # rank tests of a small shard: 12.5k 1.210 vs 1.218 ms, 25k 2.370 vs 2.360,
        # profiles/bench/serial_r6/)
        self.overlap_pairwise = self.gpu and N >= OVERLAP_MIN_SERIES
        if self.gpu:
            # graph-tick ring state: a ring of pinned sources, so a copy still in flight
            # (pipelined ticks, at most two ahead) never sees the next tick's values
            self._state_ring = torch.zeros((4, 8), dtype=torch.int32).pin_memory()
            self._state_k = 0
            self._state_dev = torch.zeros(8, dtype=torch.int32, device=self.device)
        self._state_synced = False  # the device tick record matches the host ring (graph ticks)
        # doorbell (enable_doorbell): graph ticks enqueued ahead wait for the host's counter
        self._bell: Optional[torch.Tensor] = None
        self._bell_dev: Optional[torch.Tensor] = None
        self._bell_n = 0
        # cached Holt-Winters model (refit_every > 1): state after the last refit / update
        self.refit_every = max(1, int(spec.refit_every))
        self._cache: Optional[Dict] = None
        self._new_pts = 0          # points graduated into the history since the state was advanced
        self.last_refit = True     # whether the last score() refit the model

    def refresh_thresholds(self) -> None:
        """Per-point thresholds of the full and the lowered (pairwise) band for the
        window of P*W points (models/detect.py effective_thresholds); call again
        after changing ``threshold`` / ``bound``."""
        C = self.spec.pods * self.spec.window
        self.thr_full, self.thr_low = det_ref.effective_thresholds(
            self.threshold, self.bound, C, self.cfg.pairwise_scale, self.cfg.window_correction)
        self.thr_full = self.thr_full.to(self.device).contiguous()
        self.thr_low = self.thr_low.to(self.device).contiguous()

    def enable_anomaly_list(self, cap: int) -> None:
        if self.gpu:
            from ..ops import kernels as K
            self.anomalies = K.AnomalyBuffer(cap, self.device)

    # ------------------------------------------------------------------ data in
    def load_history(self, values: torch.Tensor) -> None:
        self.hist.load(values.to(self.device))
        self._cache = None

    def load_rows(self, rows: torch.Tensor, values: torch.Tensor) -> None:
        """Write the full history AND current window of some rows (a series
        joining a running shard): ``values`` ``[k, length + W]`` oldest first,
        the last W points go to the window (every pod); the ring rotation is
        resolved with two column-slice copies, no ``[k, length]`` index tensor."""
        dev = self.device
        rows = rows.to(dev, torch.long)
        v = values.to(dev, torch.float32)
        L, R, W, P = self.hist.length, self.hist.R, self.cur.W, self.cur.P
        if v.dim() != 2 or v.shape[0] != rows.numel() or v.shape[1] != L + W:
            raise ValueError(f"values must be [{rows.numel()}, {L + W}]")
        hv = v[:, :L].to(self.hist.data.dtype)
        self._cache = None  # the new rows need a fitted state: refit on the next tick
        head = self.hist.head
        n1 = min(L, R - head)
        self.hist.data[:, head:head + n1].index_copy_(0, rows, hv[:, :n1])
        if L > n1:
            self.hist.data[:, :L - n1].index_copy_(0, rows, hv[:, n1:])
        for a in range(W):  # age a (0 = newest) sits in slot (ticks - 1 - a) mod W
            slot = (self.cur.ticks - 1 - a) % W
            col = v[:, L + W - 1 - a:L + W - a]
            for p in range(P):
                self.cur.data[:, p * W + slot:p * W + slot + 1].index_copy_(0, rows, col)

    def set_baseline(self, values: torch.Tensor) -> None:
        self.base.copy_(values.to(self.device, torch.float32))

    def _refresh_horizons(self, stable: bool = False) -> None:
        h = self.cur.horizons()
        if self.gpu:
            # The H2D copy runs when the stream reaches it, possibly after the host has moved
            # on to the next tick (pipelined ticks): its pinned source must not be rewritten
            # with other values while in flight.  Once the window is full the horizons only
            # depend on the slot, so each slot has its own pinned source (same bytes every
            # time); warm-up ticks copy from a fresh pinned buffer.
            # Eager ticks (not `stable`) in that steady state point `horizons` at the slot's
            # row of a device table instead: no per-tick copy at all.  A HIP-graph tick
            # (`stable`) needs the one buffer its capture baked in.
            W = self.cur.W
            if self.cur.ticks >= W:
                if self._h_slots is None:
                    self._h_slots = torch.empty((W, h.shape[0]), dtype=torch.int32).pin_memory()
                    for s in range(W):
                        self._h_slots[s].copy_(torch.from_numpy(self.cur.horizons(W + s)))
                    self._h_dev = self._h_slots.to(self.device)
                if not stable:
                    self.horizons = self._h_dev[self.cur.ticks % W]
                    return
                src = self._h_slots[self.cur.ticks % W]
            else:
                src = torch.from_numpy(h).pin_memory()
            self._h_buf.copy_(src, non_blocking=True)
            self.horizons = self._h_buf
        else:
            self.horizons.copy_(torch.from_numpy(h))

    def ingest_tick(self, newv: torch.Tensor, newb: Optional[torch.Tensor] = None) -> None:
        self._state_synced = False  # an eager tick moves the ring behind the device record's back
        self._ingest_tick(newv, newb)

    def _ingest_tick(self, newv: torch.Tensor, newb: Optional[torch.Tensor] = None) -> None:
        """``newv``: ``[N, P]`` float32 current-pod values on the shard's device;
        ``newb`` (optional, same shape): baseline-pod values streamed into the
        baseline window at the same slot (continuous canary).  The evicted
        slot's pod-mean graduates into the history: the baseline pods' when a
        baseline stream is given (the model tracks the stable version, never
        the canary it judges), else the current pods'."""
        graduate = self.cur.ticks >= self.cur.W
        if self.gpu:
            from ..ops import kernels as K
            K.tick_ingest(self.hist.data, self.hist.next_col(), self.cur.data, self.cur.P, self.cur.W,
                          self.cur.slot(), newv, graduate=graduate,
                          base=self.base if newb is not None else None, newb=newb,
                          zero=self.app_stats.view(-1))
            self._stats_zeroed = True  # the tick's per-app counters were cleared by the same launch
            self.cur.ticks += 1
        else:
            old_b = None
            if newb is not None:
                cols = torch.arange(self.cur.P, device=self.device) * self.cur.W + self.cur.slot()
                ob = self.base[:, cols]
                ok = ~torch.isnan(ob)
                cnt = ok.sum(1)
                old_b = torch.where(cnt > 0, torch.where(ok, ob, torch.zeros_like(ob)).sum(1) / cnt.clamp(min=1),
                                    torch.full_like(cnt, float("nan"), dtype=torch.float32))
                self.base[:, cols] = newb.float()
            old = self.cur.push_(newv)
            if old_b is not None:
                old = old_b  # canary: the baseline (stable-version) pods graduate into the history
            if graduate:
                self.hist.data[:, self.hist.next_col()] = old.to(self.hist.data.dtype)
        if graduate:
            if self.hist.length == self.hist.R:
                self._new_pts += 1   # the window slides: the cached state can absorb the point
            else:
                self._cache = None   # the window grows (padding / phases change): refit
            self.hist.advance(1)
        self._refresh_horizons()

    # ------------------------------------------------------------------ graph tick
    def enable_doorbell(self) -> None:
        """Graph ticks start by waiting for a doorbell (ops/csrc/ingest.hip
        ``tick_advance_kernel``): a tick can be enqueued before its input is released and
        starts a PCIe write after :meth:`ring` instead of a graph launch after it.  Every
        graph replay must be matched by exactly one :meth:`ring`."""
        if not self.gpu or self._bell is not None:
            return
        self._bell = torch.zeros(1, dtype=torch.int32).pin_memory()
        self._bell_dev = torch.zeros(2, dtype=torch.int32, device=self.device)
        self._bell_n = 0
        self._graphs.clear()  # recaptured with the doorbell wait

    def ring(self) -> None:
        """Release the next enqueued graph tick (doorbell mode)."""
        self._bell_n += 1
        self._bell[0] = self._bell_n

    def doorbell_timeouts(self) -> int:
        """Doorbell waits that gave up (one device sync); 0 when every replay was rung."""
        return 0 if self._bell_dev is None else int(self._bell_dev[1].item())

    def graph_ready(self) -> bool:
        """The steady state a captured tick assumes: GPU, full ring (head
        advances by one per tick), warm window (every tick graduates), the
        Holt-Winters paths that read the ring head from the device (variants 4 / 5, and 6
        at the short seasons), no anomaly list."""
        return (self.gpu and self.mode == sm_ref.MODE_HW and self.refit_every == 1
                and self.hist.length == self.hist.R
                and self.cur.ticks >= self.cur.W and self.anomalies is None
                and getattr(self, "_hw_variant", None) in (4, 5, 6) and bool(self.out))

    def tick_graph(self, newv: torch.Tensor, newb: Optional[torch.Tensor] = None,
                   post=None) -> Dict[str, torch.Tensor]:
        """``ingest_tick`` + ``score`` as ONE HIP-graph replay with no host-to-device copy.

        The graph (captured on the first steady-state call) holds a tick-advance
        kernel, the ingest kernel (which also clears the app counters), the rank
        tests and the Holt-Winters fit + deferred detection.  The ring state
        (hist column, window slot, head) lives in a device int32 record that the
        advance kernel steps by one tick at the start of every replay, and the
        forecast horizons of the new slot are copied from a device table by the
        same kernel; the host only mirrors the ring bookkeeping.  The record is
        written from the host once, when the graph path (re)starts after eager
        ticks.  Falls back to the eager calls until :meth:`graph_ready`.
        ``newv`` / ``newb``: one of at most two buffer sets (each set's addresses are baked
        into its own graph: a double-buffered input whose next tick is copied while this
        one runs).  ``post`` (optional, called once, inside the
        capture): the tick's own tail -- the node health collective and the copy of the
        health table to pinned host memory -- so one replay is the whole GPU side of the
        tick; on the eager ticks before capture the caller runs its tail itself (the
        return value's ``"post_in_graph"`` says which happened)."""
        if not self.graph_ready():
            self.ingest_tick(newv, newb)
            out = self.score()
            out["post_in_graph"] = False
            return out
        io = (newv.data_ptr(), None if newb is None else newb.data_ptr())
        hit = self._graphs.get(io)
        if hit is not None and self._state_synced and self._h_slots is not None:
            # steady state: the replay goes first and the host mirror of the ring bookkeeping
            # (nothing the replay reads) follows it, off the path from the previous tick's
            # completion to this tick's first kernel
            self._graph, self._post_in_graph, outs = hit
            self._graph.replay()
            self.hist.advance(1)
            self.cur.ticks += 1
            self._new_pts += 1
            self.horizons = self._h_buf
            self.out = dict(outs)
            self._stats_zeroed = False
            self.last_refit = True
            self.out["post_in_graph"] = self._post_in_graph
            return self.out
        if io not in self._graphs and len(self._graphs) >= 2:
            raise ValueError("tick_graph takes at most two sets of newv/newb buffers (double-buffered input)")
        W, R = self.cur.W, self.hist.R
        if self._h_slots is None:
            self._refresh_horizons()  # builds the per-slot horizon table (host + device)
        if not self._state_synced:
            # the record of the PREVIOUS tick, so that the replay's advance kernel yields this one
            st = self._state_ring[self._state_k % 4]
            self._state_k += 1
            st.zero_()
            st[1] = (self.cur.slot() - 1) % W
            st[2] = 1
            st[3] = self.hist.next_col()
            self._state_dev.copy_(st, non_blocking=True)
            self._state_synced = True
        # host mirror of the ring bookkeeping (same as ingest_tick's steady state)
        self.hist.advance(1)
        self.cur.ticks += 1
        self._new_pts += 1
        self.horizons = self._h_buf
        hit = self._graphs.get(io)
        if hit is not None:
            self._graph, self._post_in_graph, outs = hit
            self.out = dict(outs)
        else:
            from ..ops import kernels as K

            def capture(with_post: bool):
                K.reserve_graph_workspace(self.device, self.hist.data.shape[0])
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    K.tick_advance(self._state_dev, R, W, self._h_dev, self._h_buf, bell=self._bell,
                                   bell_dev=self._bell_dev)
                    K.tick_ingest(self.hist.data, 0, self.cur.data, self.cur.P, self.cur.W, 0, newv,
                                  base=self.base if newb is not None else None, newb=newb, state=self._state_dev,
                                  zero=self.app_stats.view(-1))
                    self._score_gpu(head_dev=self._state_dev[3:4])
                    if with_post:
                        post()
                return g
            g, self._post_in_graph = None, False
            if post is not None:
                try:
                    g, self._post_in_graph = capture(True), True
                except RuntimeError:  # e.g. a collective backend that cannot be captured
                    torch.cuda.synchronize()
                    g = None
            if g is None:
                g = capture(False)
            self._graph, self._graph_io = g, io
            self._graphs[io] = (g, self._post_in_graph, dict(self.out))
        self._graph.replay()
        self._stats_zeroed = False
        self.last_refit = True
        self.out["post_in_graph"] = self._post_in_graph
        return self.out

    # ------------------------------------------------------------------ scoring
    def score(self) -> Dict[str, torch.Tensor]:
        if not self._stats_zeroed:
            self.app_stats.zero_()
        self._stats_zeroed = False
        cached = self._use_cache()
        self.last_refit = not cached
        if self.gpu:
            out = self._score_cached_gpu() if cached else self._score_gpu()
        else:
            out = self._score_cpu(cached)
        if self._cache is not None:
            self._cache["since"] = 0 if not cached else self._cache["since"] + 1
        return out

    # ------------------------------------------------------------------ model cache
    def cache_supported(self) -> bool:
        from ..ops import kernels as K
        return (self.refit_every > 1 and self.mode == sm_ref.MODE_HW
                and (not self.gpu or self.spec.season >= K.HW_STATE_MIN_M))

    def _use_cache(self) -> bool:
        c = self._cache
        return (c is not None and self.cache_supported() and c["since"] + 1 < self.refit_every
                and self.hist.length == self.hist.R and self._new_pts <= self.hist.R)

    def _rank_tests_main(self):
        """Pairwise tests on the current stream (cached ticks: nothing to overlap)."""
        from ..ops import kernels as K
        cfg = self.cfg
        if self.pw_mode == pw_ref.PW_NONE:
            return None
        self.pw_out = K.rank_tests(self.base, self.cur.data, self.pw_mode, cfg.pairwise_threshold,
                                   cfg.min_mann_white, cfg.min_wilcoxon, cfg.min_kruskal,
                                   want_pvals=True, out=self.pw_out, pods=(self.cur.P, self.cur.P),
                                   min_friedman=cfg.min_friedman)
        return self.pw_out["differs"]

    def _detect_spec(self, differs):
        from ..ops import kernels as K
        cfg = self.cfg
        return K.DetectSpec(horizons=self.horizons, threshold=self.thr_full, bound=self.bound,
                            min_lower=self.min_lower, cur=self.cur.data, differs=differs,
                            pw_scale=cfg.pairwise_scale, min_valid=cfg.min_historical_points,
                            want_band=self.spec.want_band, app_id=self.app_id, app_stats=self.app_stats,
                            anomalies=self.anomalies, max_horizon=self.cur.W, threshold_low=self.thr_low,
                            pw_min_points=cfg.pairwise_min_points,
                            shift_threshold=cfg.pairwise_shift, shift_min_points=cfg.pairwise_shift_min_points,
                            shift_one_step=cfg.pairwise_shift_one_step,
                            base_mean=self.pw_out["base_mean"] if differs is not None else None,
                            horizon_variance=cfg.horizon_variance)

    def _refresh_cache_gpu(self) -> None:
        """After a refit: the full state of the fitted model (hw_state.hip)."""
        from ..ops import kernels as K
        if not self.cache_supported() or self.hist.length != self.hist.R:
            self._cache = None
            return
        h = self.hist
        prev = self._cache["state"] if self._cache is not None else None
        st = K.hw_state(h.data, h.head, h.length, self.spec.season, self.grid, self.out["best"], state=prev)
        self._cache = {"state": st, "t_last": st["Tp"] - 1, "since": 0,
                       "sigma": self.out["sigma"], "best": self.out["best"]}
        self._new_pts = 0

    def _score_cached_gpu(self) -> Dict[str, torch.Tensor]:
        from ..ops import kernels as K
        c, h = self._cache, self.hist
        differs = self._rank_tests_main()
        spec = self._detect_spec(differs)
        if self.anomalies is not None:
            self.anomalies.reset()
        npts = self._new_pts
        col0 = (h.head + h.length - npts) % h.R
        self.out = K.hw_update_detect(h.data, col0, npts, c["t_last"], self.spec.season, self.grid, c["best"],
                                      c["state"], c["sigma"], c["state"]["nvalid"], spec, out=self.out)
        c["t_last"] += npts
        self._new_pts = 0
        return self.out

    def _score_gpu(self, head_dev: Optional[torch.Tensor] = None) -> Dict[str, torch.Tensor]:
        from ..ops import kernels as K
        cfg = self.cfg
        differs = None
        # Holt-Winters: the rank tests run on a side stream concurrently with the fit,
        # whose band/verdict epilogue is deferred until both are done
        overlap = self.pw_mode != pw_ref.PW_NONE and self.mode == sm_ref.MODE_HW and self.overlap_pairwise
        main = torch.cuda.current_stream(self.device)
        if self.pw_mode != pw_ref.PW_NONE:
            def _rank():
                return K.rank_tests(self.base, self.cur.data, self.pw_mode, cfg.pairwise_threshold,
                                    cfg.min_mann_white, cfg.min_wilcoxon, cfg.min_kruskal,
                                    want_pvals=True, out=self.pw_out, pods=(self.cur.P, self.cur.P),
                                    min_friedman=cfg.min_friedman)
            if overlap:
                if self._side is None:
                    self._side = torch.cuda.Stream(self.device)
                self._side.wait_stream(main)  # after this tick's ingest
                with torch.cuda.stream(self._side):
                    self.pw_out = _rank()
            else:
                self.pw_out = _rank()
            differs = self.pw_out["differs"]
        spec = K.DetectSpec(horizons=self.horizons, threshold=self.thr_full, bound=self.bound,
                            min_lower=self.min_lower, cur=self.cur.data, differs=differs,
                            pw_scale=cfg.pairwise_scale, min_valid=cfg.min_historical_points,
                            want_band=self.spec.want_band, app_id=self.app_id, app_stats=self.app_stats,
                            anomalies=self.anomalies, max_horizon=self.cur.W, threshold_low=self.thr_low,
                            pw_min_points=cfg.pairwise_min_points,
                            shift_threshold=cfg.pairwise_shift, shift_min_points=cfg.pairwise_shift_min_points,
                            shift_one_step=cfg.pairwise_shift_one_step,
                            base_mean=self.pw_out["base_mean"] if differs is not None else None,
                            horizon_variance=cfg.horizon_variance)
        if self.anomalies is not None:
            self.anomalies.reset()
        h = self.hist
        if self.mode is not None:
            self.out = K.smoothing_fit(h.data, h.head, h.length, self.mode, self.spec.season, self.grid,
                                       spec, out=self.out, head_dev=head_dev, defer_detect=overlap,
                                       detect_after=self._side if overlap else None)
            self._hw_variant = K.last_hw_variant
            if overlap and K.last_detect_deferred:
                main.wait_stream(self._side)
                Tp = K.smoothing_geometry(self.mode, h.length, self.spec.season)[0]
                K.hw_detect_deferred(self.out, spec, Tp, self.spec.season, grid=self.grid)
            if self.refit_every > 1 and head_dev is None:
                self._refresh_cache_gpu()
        elif self.algorithm in ("moving_average_all", "moving_average"):
            length = h.length
            head = h.head
            if self.algorithm == "moving_average" and cfg.ma_window < length:
                head = (h.head + length - cfg.ma_window) % h.R
                length = cfg.ma_window
            self.out = K.window_stats(h.data, head, length, spec, out=self.out)
        elif self.algorithm == "seasonal_decompose":
            self.out = K.decompose_score(h.data, h.head, h.length, self.spec.season, spec, out=self.out)
        else:
            raise ValueError(f"algorithm {self.algorithm!r} is not a streaming univariate scorer")
        return self.out

    def _score_cpu(self, cached: bool = False) -> Dict[str, torch.Tensor]:
        cfg = self.cfg
        y = self.hist.logical().float()
        differs = None
        if self.pw_mode != pw_ref.PW_NONE:
            res = pw_ref.rank_tests(self.base, self.cur.data, pods=(self.cur.P, self.cur.P))
            differs = pw_ref.pairwise_differs(res, self.pw_mode, cfg.pairwise_threshold, cfg.min_mann_white,
                                              cfg.min_wilcoxon, cfg.min_kruskal, cfg.min_friedman)
            self.pw_out = {"differs": differs.to(torch.uint8),
                           "pvals": torch.stack([res.p_mw, res.p_wilcoxon, res.p_kruskal], 1).float(),
                           "friedman": torch.stack([res.p_friedman, res.n_blocks], 1).float()}
        h = self.horizons.long()
        valid_hist = (~torch.isnan(y)).sum(1)
        if cached:
            c = self._cache
            params = self.grid.cpu()[c["best"].long()]
            st = c["state"]
            if self._new_pts:
                sm_ref.hw_update(st, y[:, y.shape[1] - self._new_pts:], params)
            self._new_pts = 0
            f = sm_ref.hw_state_forecast(st, h)
            n_valid = c["n_valid"]
            extra = {"level": st.level, "trend": st.trend, "sigma": c["sigma"], "best": c["best"]}
            sigma = c["sigma"]
            if cfg.horizon_variance:
                sigma = c["sigma"][:, None] * det_ref.horizon_sigma_factor(params, self.mode, self.spec.season, h)
        elif self.algorithm == "seasonal_decompose":
            from ..models import decompose as dec_ref
            fc = dec_ref.decompose_forecast(y, self.spec.season)
            f = dec_ref.forecast_decomposition(fc, h)
            sigma, n_valid = fc.sigma, fc.n_valid
            extra = {"level": fc.level, "slope": fc.slope, "sigma": fc.sigma}
        elif self.mode is not None:
            fit = sm_ref.fit_smoothing(y, self.mode, self.grid.cpu(), m=self.spec.season)
            f = sm_ref.forecast(fit, h)
            n_valid = fit.n_valid
            extra = {"level": fit.level, "trend": fit.trend, "sigma": fit.sigma, "best": fit.best.int()}
            sigma = fit.sigma
            if cfg.horizon_variance:
                params = self.grid.cpu()[fit.best.long()]
                sigma = fit.sigma[:, None] * det_ref.horizon_sigma_factor(params, self.mode, self.spec.season, h)
            if self.cache_supported() and self.hist.length == self.hist.R:
                self._cache = {"state": sm_ref.HwState(level=fit.level.clone(), trend=fit.trend.clone(),
                                                       season=fit.season.clone(), t_last=fit.t_len - 1,
                                                       m=self.spec.season),
                               "since": 0, "sigma": fit.sigma, "best": fit.best.int(), "n_valid": fit.n_valid}
                self._new_pts = 0
            else:
                self._cache = None
        else:
            win = cfg.ma_window if self.algorithm == "moving_average" else None
            st = ma_ref.window_stats(y, win)
            f = st.mean[:, None].expand(-1, h.shape[0])
            sigma = st.std
            n_valid = st.count
            extra = {"mean": st.mean, "std": st.std}
        ok = n_valid >= cfg.min_historical_points
        sigma1 = extra["sigma"] if "sigma" in extra else extra["std"]  # one-step (the mean-shift rule's spread)
        d = det_ref.detect(f, sigma, self.cur.data, self.thr_full, self.bound, self.min_lower,
                           differs=differs, pairwise_scale=cfg.pairwise_scale, model_ok=ok,
                           threshold_low=self.thr_low, pw_min_points=cfg.pairwise_min_points,
                           shift_threshold=cfg.pairwise_shift, shift_min_points=cfg.pairwise_shift_min_points,
                           base_mean=torch.nanmean(self.base.float(), 1) if differs is not None else None,
                           shift_sigma=sigma1 if cfg.pairwise_shift_one_step else None)
        v = d.verdict.long()
        self.app_stats.index_put_((self.app_id.long(), torch.zeros_like(v)), (v == 1).int(), accumulate=True)
        self.app_stats.index_put_((self.app_id.long(), torch.ones_like(v)), (v >= 0).int(), accumulate=True)
        del valid_hist
        verdict = d.verdict
        if self._verdict_out is not None:
            verdict = self._verdict_out.copy_(d.verdict)
        self.out = dict(extra, forecast=f, upper=d.upper, lower=d.lower, count=d.count,
                        verdict=verdict, score=d.score)
        return self.out


def synthetic_params(N: int, device, seed: int = 0, rows: Optional[Tuple[int, int]] = None) -> Dict[str, torch.Tensor]:
    """Per-series parameters of the synthetic seasonal model: level, daily
    amplitude, phase, linear trend (each ``[N, 1]``).  ``rows = (s, e)``: only
    global series ``s .. e-1`` of the ``N`` (a rank's shard gets exactly the
    parameters the one-rank run gives those series)."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    lvl = torch.rand((N, 1), generator=g, device=device) * 95 + 5
    amp = (torch.rand((N, 1), generator=g, device=device) * 0.25 + 0.05) * lvl
    ph = torch.rand((N, 1), generator=g, device=device) * 6.283
    tr = (torch.rand((N, 1), generator=g, device=device) - 0.5) * 1e-4 * lvl
    out = {"lvl": lvl, "amp": amp, "ph": ph, "tr": tr}
    if rows is not None:
        out = {k: v[rows[0]:rows[1]].contiguous() for k, v in out.items()}
    return out


NOISE_CHUNK = 8192  # synthetic noise is drawn per block of this many GLOBAL series


def global_randn(shape_fn, n: int, row0: int, seed: int, device, dim: int = 0) -> torch.Tensor:
    """Standard normal draws for global series ``row0 .. row0+n-1`` along ``dim``:
    block ``c`` of :data:`NOISE_CHUNK` global series comes from its own generator
    (``seed`` + c), so any shard of the series sees the draws the whole set
    sees.  ``shape_fn(rows)`` gives the block shape for ``rows`` series."""
    parts = []
    c0, c1 = row0 // NOISE_CHUNK, (row0 + n - 1) // NOISE_CHUNK if n else row0 // NOISE_CHUNK - 1
    for c in range(c0, c1 + 1):
        g = torch.Generator(device=device)
        g.manual_seed(seed * 1_000_003 + c)
        blk = torch.randn(shape_fn(NOISE_CHUNK), generator=g, device=device)
        lo = max(row0, c * NOISE_CHUNK) - c * NOISE_CHUNK
        hi = min(row0 + n, (c + 1) * NOISE_CHUNK) - c * NOISE_CHUNK
        parts.append(blk.narrow(dim, lo, hi - lo))
    if not parts:
        return torch.empty(shape_fn(0), device=device)
    return torch.cat(parts, dim) if len(parts) > 1 else parts[0].contiguous()


def synthetic_eval(params: Dict[str, torch.Tensor], t0: int, T: int, season: int, noise_seed: Optional[int],
                   dtype=torch.float32, chunk: int = NOISE_CHUNK, noise: float = 0.03, row0: int = 0) -> torch.Tensor:
    """Values of the synthetic model at times ``t0 .. t0+T-1`` → ``[N, T]``;
    i.i.d. Gaussian noise of ``noise * level`` unless ``noise_seed`` is None.
    ``row0``: global index of the first series (noise is a function of the
    global series index, see :func:`global_randn`)."""
    lvl = params["lvl"]
    N, dev = lvl.shape[0], lvl.device
    out = torch.empty((N, T), dtype=dtype, device=dev)
    t = torch.arange(t0, t0 + T, device=dev, dtype=torch.float32)
    for s in range(0, N, chunk):
        e = min(N, s + chunk)
        y = lvl[s:e] + params["tr"][s:e] * t + params["amp"][s:e] * torch.sin(2 * np.pi * t / season + params["ph"][s:e])
        if noise_seed is not None:
            y = y + global_randn(lambda r: (r, T), e - s, row0 + s, noise_seed, dev) * (noise * lvl[s:e])
        out[s:e] = y.to(dtype)
    return out


def synthetic_history(N: int, T: int, season: int, device, seed: int = 0, dtype=torch.float32,
                      chunk: int = NOISE_CHUNK) -> torch.Tensor:
    """Seasonal synthetic series (level, daily seasonality, slight trend, noise)
    generated on ``device`` in chunks; returns ``[N, T]`` in ``dtype``.
    Continue a series with ``synthetic_eval(synthetic_params(N, dev, seed), T, ...)``."""
    return synthetic_eval(synthetic_params(N, device, seed), 0, T, season, seed + 1_000_003, dtype, chunk)
