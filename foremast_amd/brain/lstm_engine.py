"""Streaming LSTM-autoencoder scoring for one shard (BASELINE configs 3 and 5).

Per tick:

1. ingest one new point per (series, metric) into the per-metric HBM rings;
2. one data-parallel training step of the shared LSTM-AE on a minibatch of
   history windows sampled from this rank's shard (gradient all-reduce over
   RCCL, :mod:`foremast_amd.parallel.dp`);
3. repack the updated weights into MFMA fragment order on the device;
4. score every series' latest window with the fused kernel (bf16, or fp8
   e4m3 for the multivariate service-mesh config) → reconstruction z-score
   → verdict → per-app counters.

Per-series normalisation statistics (mean/std per metric) come from the
``window_stats`` kernel over the history ring and are refreshed every
``restat_every`` ticks.

Detection is calibrated per series: one shared model reconstructs a calm,
noise-dominated series far better than a noisy one, so a single global
error threshold flags the noisy series and misses regressions on the calm
ones.  :meth:`LstmShard.calibrate` scores ``cal_windows`` history windows of
EVERY series with the scoring kernel and keeps each series' healthy error
level ``mu_i``; the dispersion is pooled as a relative spread ``rho`` of
``err / mu_i`` over all windows (ranks combine it with one all-reduce), so
``z_i = (err - mu_i) / (rho * mu_i)``.  The verdict z-score is the smaller
of ``z_i`` and the global one (``(err - mu) / sigma``, errors being in
series-std units): a window is anomalous only when it is unusual for its
series AND in absolute terms.  Measured on 20k healthy + 200 x3-regressed
multivariate entities (fp8), thr 4: per-series alone flags 605 healthy
entities, global alone 263, both 27, every regression caught by each.  Each
tick the kernel's epilogue moves ``mu_i`` toward the series' errors that lie
within ``CAL_GATE`` of its level (``cal_ewma``), tracking the continuously
trained model without absorbing a regression that builds up over ticks.

Level term: the autoencoder scores the *shape* of a z-scored 32-point window,
so a level shift of a few noise sigmas inside the daily swing is weak evidence
for it (round-2 sweep: +3 sigma recall 0.24).  Each tick ``lstm_level``
(csrc/lstm.hip) computes, per (series, feature), the mean of the newest 8
samples minus its forecast from the earlier days the ring holds (<= 7): the
centred (up to) 32-point mean around the same minutes of each day, extrapolated to
today by least squares over the days (a linear trend across days cancels),
divided by that statistic's own spread — calibrated on the series' history as
the RMS of the statistic at ``level_cal`` earlier offsets (:meth:`calibrate`).  A window is anomalous when the AE z-score OR any
feature's ``|level z|`` exceeds its threshold (``level_threshold``; the
epilogue also keeps such windows out of the calibration refresh).
"""

from __future__ import annotations

import os
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from ..ingest.ringbuffer import HistoryRing
from ..models.lstm_ae import LSTMAutoencoder
from ..parallel import comm
from ..parallel.dp import DPTrainer


CAL_GATE = 2.0  # csrc/lstm.hip: errors above 2 series-sigma do not refresh the calibration


class LstmShard:
    def __init__(self, n_series: int, ring_len: int, n_features: int, window: int = 32, hidden: int = 64,
                 fp8: bool = False, device="cuda", app_id: Optional[torch.Tensor] = None, n_apps: int = 1,
                 threshold: float = 4.0, train_batch: int = 4096, lr: float = 1e-3, restat_every: int = 16,
                 seed: int = 0, dtype=torch.bfloat16, fused_train: bool = True, cal_windows: int = 16,
                 cal_ewma: float = 1.0 / 32, dp_overlap: bool = True, season: int = 1440,
                 level_points: int = 8, level_threshold: Optional[float] = 5.5, level_cal: int = 64) -> None:
        self.n, self.R, self.F, self.T = n_series, ring_len, n_features, window
        self.device = torch.device(device)
        self.gpu = self.device.type == "cuda"
        self.rings: List[HistoryRing] = [HistoryRing(n_series, ring_len, dtype, self.device)
                                         for _ in range(n_features)]
        torch.manual_seed(seed)
        self.model = LSTMAutoencoder(n_features, hidden).to(self.device)
        grad_fn = None
        if self.gpu and fused_train and train_batch % 32 == 0:
            from ..ops.lstm_train import FusedLstmGrad
            self.fg = FusedLstmGrad(train_batch, window, n_features, self.device)
            grad_fn = self.fg.grads
        self.fused_train = grad_fn is not None
        self.trainer = DPTrainer(self.model, lr=lr, grad_fn=grad_fn, overlap=dp_overlap)
        self.dtype = dtype
        # rows training samples are drawn from (None: every row); the resident monitor
        # (brain/lstm_monitor.py) keeps free rows out of training
        self.live: Optional[torch.Tensor] = None
        self.fp8 = fp8
        self.train_batch = train_batch
        self.threshold = threshold
        self.restat_every = restat_every
        self.app_id = app_id if app_id is not None else torch.zeros(n_series, dtype=torch.int32,
                                                                    device=self.device)
        self.app_stats = torch.zeros((max(n_apps, 1), 2), dtype=torch.int32, device=self.device)
        self.mean = torch.zeros(n_series, n_features, device=self.device)
        self.std = torch.ones(n_series, n_features, device=self.device)
        self.rstd = torch.ones(n_series, n_features, device=self.device)
        self.mu, self.sigma = 0.0, 1.0
        self.cal_windows, self.cal_ewma = cal_windows, cal_ewma
        self.cal: Optional[torch.Tensor] = None  # [n, 2] (mu_i, 1 / (rho * mu_i)) after calibrate()
        self.rho = 1.0
        if level_points != 8:
            raise ValueError("level_points: the level kernel averages the newest 8 points")
        self.season, self.level_points, self.level_cal = int(season), int(level_points), int(level_cal)
        self.level_threshold = level_threshold
        self.lvl_sig: Optional[torch.Tensor] = None  # [n, F] spread of the level statistic after calibrate()
        self._zl: Optional[torch.Tensor] = None
        self.ticks = 0
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(seed + 1)
        self.packed = None
        self.out: Dict[str, torch.Tensor] = {}
        self._ar = torch.arange(window, device=self.device)
        self._det = None
        self._side = None
        self._ws: Dict[str, torch.Tensor] = {}
        self._all = torch.arange(n_series, device=self.device)
        self._zero_off = torch.zeros(n_series, dtype=torch.long, device=self.device)
        # whole-tick HIP graph (tick_graph): ring positions travel in a device record
        # [append column, head after the append] that the replay steps by one tick; the
        # host writes it only when the rings moved without it (eager ticks, reloads)
        self.graph_on = self.gpu and os.environ.get("FOREMAST_LSTM_GRAPH", "1") != "0"
        self._graph = None
        self._graph_key = None
        self.graph_replays = 0
        self._grec_last = None  # positions the device record holds after the last graph tick
        self._grec_k = 0
        if self.gpu:
            # a ring of pinned sources: a re-sync's copy may still be in flight at the next one
            self._grec_host = torch.zeros((4, 2), dtype=torch.int32).pin_memory()
            self._grec_dev = torch.zeros(2, dtype=torch.int32, device=self.device)

    # ------------------------------------------------------------------ rows (resident monitor)
    def grow(self, capacity: int) -> None:
        """Re-allocate for ``capacity`` rows, keeping every row's ring, statistics
        and calibration (the model and optimizer are untouched)."""
        n, dev = self.n, self.device
        if capacity <= n:
            return
        for f, ring in enumerate(self.rings):
            new = HistoryRing(capacity, self.R, self.dtype, dev)
            new._store[:n].copy_(ring._store)
            new.state.head, new.state.length = ring.head, ring.length
            self.rings[f] = new

        def ext(t, fill):
            out = torch.full((capacity,) + tuple(t.shape[1:]), fill, dtype=t.dtype, device=dev)
            out[:n].copy_(t)
            return out
        self.mean, self.std, self.rstd = ext(self.mean, 0.0), ext(self.std, 1.0), ext(self.rstd, 1.0)
        self.app_id = ext(self.app_id, 0)
        if self.cal is not None:
            self.cal = ext(self.cal, 1.0).contiguous()
        if self.lvl_sig is not None:  # rows not calibrated yet carry no level term (z = 0)
            self.lvl_sig = ext(self.lvl_sig, float("inf")).contiguous()
        self.n = capacity
        self._all = torch.arange(capacity, device=dev)
        self._zero_off = torch.zeros(capacity, dtype=torch.long, device=dev)
        self.out = {}

    def write_rows(self, rows: torch.Tensor, values) -> None:
        """History of some rows: ``values`` F tensors ``[k, length]`` in time order,
        ending at the rings' newest sample (the ring rotation is resolved with
        two column-slice copies)."""
        rows = rows.to(self.device, torch.long)
        for f, ring in enumerate(self.rings):
            v = values[f].to(self.device, ring.data.dtype)
            L, R, head = ring.length, ring.R, ring.head
            v = v[:, -L:]
            n1 = min(L, R - head)
            ring.data[:, head:head + n1].index_copy_(0, rows, v[:, :n1])
            if L > n1:
                ring.data[:, :L - n1].index_copy_(0, rows, v[:, n1:])

    def _draw_rows(self, B: int, dtype) -> torch.Tensor:
        if self.live is None:
            return torch.randint(0, self.n, (B,), generator=self.gen, device=self.device, dtype=dtype)
        k = torch.randint(0, max(1, self.live.numel()), (B,), generator=self.gen, device=self.device)
        return self.live[k].to(dtype)

    # ------------------------------------------------------------------ data
    def load_history(self, values) -> None:
        """``values``: ``[n, T_hist, F]`` or a list of F ``[n, T_hist]`` tensors."""
        for f, ring in enumerate(self.rings):
            ring.load(values[f] if isinstance(values, (list, tuple)) else values[..., f])
        self.refresh_stats()

    def refresh_stats(self) -> None:
        """Per-series mean/std of each metric over the whole history ring
        (``window_stats`` kernel on the GPU: one HBM pass, no fp32 copy)."""
        if self.gpu:
            from ..ops import kernels as K
            if self._det is None:
                n, dev = self.n, self.device
                self._det = K.DetectSpec(horizons=torch.ones(1, dtype=torch.int32, device=dev),
                                         threshold=torch.zeros(n, device=dev),
                                         bound=torch.zeros(n, dtype=torch.int8, device=dev),
                                         min_lower=torch.zeros(n, device=dev), want_band=False)
            for f, ring in enumerate(self.rings):
                o = K.window_stats(ring.data, ring.head, ring.length, self._det, out=self._ws)
                self.mean[:, f] = o["mean"]
                self.std[:, f] = o["std"].clamp(min=1e-6)
            torch.reciprocal(self.std, out=self.rstd)
            return
        for f, ring in enumerate(self.rings):
            yf = ring.logical().float()
            self.mean[:, f] = yf.mean(1)
            self.std[:, f] = yf.std(1, unbiased=False).clamp(min=1e-6)

    def ingest_tick(self, newv: torch.Tensor) -> None:
        """``newv``: ``[n, F]`` float32."""
        for f, ring in enumerate(self.rings):
            col = ring.next_col()
            if self.gpu:
                from ..ops import kernels as K
                K.ring_append(ring.data, col, newv[:, f:f + 1])
            else:
                ring.data[:, col] = newv[:, f].to(ring.data.dtype)
            ring.advance(1)
        self.ticks += 1
        if self.ticks % self.restat_every == 0:
            self.refresh_stats()

    def _gather(self, series_idx: torch.Tensor, end_offsets: torch.Tensor) -> torch.Tensor:
        """Windows ending ``end_offsets`` samples before the newest one → ``[B, T, F]`` normalised."""
        ring0 = self.rings[0]
        L = ring0.length
        start = L - self.T - end_offsets  # logical start index
        cols = (ring0.head + start[:, None] + self._ar[None, :]) % ring0.R  # [B, T]
        feats = [ring.data[series_idx[:, None], cols].float() for ring in self.rings]
        x = torch.stack(feats, 2)  # [B, T, F]
        return ((x - self.mean[series_idx][:, None, :]) / self.std[series_idx][:, None, :]).contiguous()

    def _ring_src_dev(self, win_series: Optional[torch.Tensor] = None,
                      win_start: Optional[torch.Tensor] = None):
        """:meth:`_ring_src` with the head on the device (graph ticks): the scoring
        window starts ``length - T`` after it, sampled windows ``win_start`` after it."""
        from ..ops.lstm import RingSource
        r0 = self.rings[0]
        return RingSource(rings=[r.data for r in self.rings], start_col=r0.length - self.T, mean=self.mean,
                          rstd=self.rstd, win_series=win_series, win_start=win_start, head_dev=self._grec_dev[1:2])

    def _ring_src(self, win_series: Optional[torch.Tensor] = None, win_start: Optional[torch.Tensor] = None):
        """Kernel-side input: the kernels read the bf16 rings directly and
        z-score on the fly, so no ``[B, T, F]`` window tensor is materialised.
        Without ``win_series`` row n scores its newest ``T`` samples."""
        from ..ops.lstm import RingSource
        r0 = self.rings[0]
        return RingSource(rings=[r.data for r in self.rings], start_col=(r0.head + r0.length - self.T) % r0.R,
                          mean=self.mean, rstd=self.rstd, win_series=win_series, win_start=win_start)

    def _sample_ring_dev(self, B: int):
        """:meth:`_sample_ring` with starts as offsets from the device head (same draws)."""
        L = self.rings[0].length
        si = self._draw_rows(B, torch.int32)
        st = torch.randint(1, L - self.T + 1, (B,), generator=self.gen, device=self.device, dtype=torch.int32)
        return self._ring_src_dev(si, st)

    def _sample_ring(self, B: int):
        """``B`` random history windows as ring coordinates (two RNG launches):
        logical start in ``[1, L - T]`` → physical ``head + start`` (the kernel
        reduces it mod R); same distribution as :meth:`_sample`."""
        r0 = self.rings[0]
        L = r0.length
        si = self._draw_rows(B, torch.int32)
        if L > self.T:
            st = torch.randint(r0.head + 1, r0.head + L - self.T + 1, (B,), generator=self.gen,
                               device=self.device, dtype=torch.int32)
        else:  # too little history: every sample is the (NaN-padded) newest window
            st = torch.full((B,), (r0.head + L - self.T) % r0.R, dtype=torch.int32, device=self.device)
        return self._ring_src(si, st)

    # ------------------------------------------------------------------ train / score
    def _sample(self, B: int) -> torch.Tensor:
        L = self.rings[0].length
        si = self._draw_rows(B, torch.int64)
        off = torch.randint(0, max(1, L - self.T), (B,), generator=self.gen, device=self.device)
        return self._gather(si, off)

    def train_step(self, weight: Optional[float] = None, flags: Optional[torch.Tensor] = None,
                   timeout_s: Optional[float] = None) -> torch.Tensor:
        """One DP step on ``train_batch`` history windows of this shard.
        ``weight`` 0: no live rows — join the gradient reduction with nothing
        (see :meth:`DPTrainer.step`); ``flags``: summed in the same collective."""
        kw = dict(weight=weight, flags=flags, timeout_s=timeout_s)
        if weight is not None and weight == 0:
            return self.trainer.step(None, grad_fn=lambda m, _w: torch.zeros((), device=self.device), **kw)
        if self.fused_train:
            return self.trainer.step(self._sample_ring(self.train_batch), **kw)
        return self.trainer.step(self._sample(self.train_batch), **kw)

    def calibrate(self, n: int = 4096, rows: Optional[torch.Tensor] = None) -> None:
        """Calibrate the verdict threshold on healthy history (untimed, once and
        then on a slow cadence).

        Global: reconstruction-error mean/std over ``n`` random history windows
        per rank, combined across ranks (one 3-float all-reduce).  Per series
        (``cal_windows > 0``): every series' ``cal_windows`` windows at evenly
        spaced history offsets → ``mu_i`` (mean without the largest, so one
        unusual day does not inflate it) and the pooled relative spread
        ``rho``.  On the GPU the windows are scored by the SAME fused kernel
        (and precision: bf16, or fp8 e4m3) that scores the ticks, so the
        calibration includes the scoring path's quantisation noise.

        ``rows``: calibrate only these rows' ``mu_i`` (series that joined a
        running monitor); the global level and ``rho`` are still re-estimated
        over the live rows with the same collectives on every rank."""
        if self.live is not None and self.live.numel() == 0:  # nothing live here: join the reductions
            e = torch.zeros(0, dtype=torch.float64, device=self.device)
        else:
            e = self._calib_errors(self._sample_ring(n) if self.gpu else None, n)
        e = e[torch.isfinite(e)]
        mom = torch.stack([e.sum(), (e * e).sum(), torch.tensor(float(e.numel()), dtype=torch.float64,
                                                                device=e.device)])
        self._all_reduce(mom)
        s1, s2, cnt = mom.tolist()
        if cnt > 0:
            self.mu = s1 / cnt
            self.sigma = max(s2 / cnt - self.mu * self.mu, 0.0) ** 0.5 + 1e-12
        if self.cal_windows <= 0:
            self.cal = None
            return
        K, L, R = self.cal_windows, self.rings[0].length, self.rings[0].R
        span = max(L - self.T, 1)
        offs = [(k * span) // K for k in range(K)]  # logical window starts, oldest first
        sel = self._all if rows is None else rows.to(self.device, torch.long)
        nr = int(sel.numel())
        if self.gpu:
            head = self.rings[0].head
            si = sel.to(torch.int32).repeat(K)
            st = torch.tensor([(head + o) % R for o in offs], dtype=torch.int32,
                              device=self.device).repeat_interleave(nr)
            ek = self._calib_errors(self._ring_src(si, st), K * nr).view(K, nr)
        else:
            ek = torch.stack([self._calib_errors(self._gather(sel, torch.full_like(
                sel, L - self.T - o)), nr) for o in offs])
        ek = torch.where(torch.isfinite(ek), ek, torch.nan)
        srt = ek.sort(0).values  # NaN last
        ok = torch.isfinite(srt)
        cnt_i = ok.sum(0)
        keep = ok & (torch.arange(K, device=ek.device)[:, None] < (cnt_i - 1).clamp(min=1)[None, :])
        mu_i = torch.where(keep, srt, 0.0).sum(0) / keep.sum(0).clamp(min=1)
        floor = max(self.mu * 1e-3, 1e-12)
        mu_i = torch.where(cnt_i > 0, mu_i, self.mu).clamp(min=floor)
        r = ek / mu_i[None, :] - 1.0
        r = r[torch.isfinite(r)]
        mom = torch.stack([r.sum(), (r * r).sum(), torch.tensor(float(r.numel()), dtype=torch.float64,
                                                                device=r.device)])
        self._all_reduce(mom)
        r1, r2, rc = mom.tolist()
        m1 = r1 / max(rc, 1.0)
        if rc > 0:
            self.rho = max((max(r2 / max(rc, 1.0) - m1 * m1, 0.0)) ** 0.5, 1e-6)
        new = torch.stack([mu_i, 1.0 / (self.rho * mu_i)], 1).float()
        if rows is None or self.cal is None:
            full = torch.ones((self.n, 2), dtype=torch.float32, device=self.device)
            full[sel] = new
            self.cal = full.contiguous()
        else:
            self.cal[sel] = new
        self.calibrate_level(rows)

    # ------------------------------------------------------------------ level term
    @property
    def LVL_E(self) -> int:  # extra minutes each side of the earlier days' windows (ops/lstm.py)
        from ..ops.lstm import level_extension
        return level_extension(self.season)

    def _level_geometry(self):
        r0 = self.rings[0]
        L, m, avail = self.level_points, self.season, r0.length
        back_max = avail - (L + self.LVL_E) - m  # offsets keep at least one earlier day behind them
        if self.level_threshold is None or back_max < L:
            return None
        step = max(L, min(back_max, m) // max(self.level_cal, 1))
        K = max(1, min(self.level_cal, back_max // step))
        return (r0.head + avail - 1) % r0.R, avail, K, step

    def _level_stat_cpu(self, back: int) -> torch.Tensor:
        """The level statistic ``[n, F]`` ending ``back`` samples before the newest
        (same definition as ``lstm_level_kernel``): the newest ``L`` points' mean minus
        its least-squares extrapolation over the earlier days' centred 32-point means."""
        r0 = self.rings[0]
        L, E, m, avail = self.level_points, self.LVL_E, self.season, r0.length
        W = L + 2 * E
        D = min(7, (avail - back - (L + E)) // m)
        out = torch.full((self.n, self.F), float("nan"), device=self.device)
        if D < 1:
            return out
        p = torch.arange(W, device=self.device)
        d = torch.arange(D + 1, device=self.device)
        logical = avail - 1 - back - (L + E - 1) + p[None, :] - d[:, None] * m  # [D+1, W]
        cols = (r0.head + logical) % r0.R
        fd = d[1:].to(torch.float32)
        for f, ring in enumerate(self.rings):
            x = ring.data[:, cols.reshape(-1)].float().view(self.n, D + 1, W)
            today = torch.nanmean(x[:, 0, E:E + L], 1)
            b = torch.nanmean(x[:, 1:], 2)  # [n, D]
            ok = torch.isfinite(b)
            w = ok.float()
            s0 = w.sum(1)
            s1 = (w * fd).sum(1)
            s2 = (w * fd * fd).sum(1)
            bz = torch.where(ok, b, 0.0)
            sb = bz.sum(1)
            sdb = (bz * fd).sum(1)
            dbar = s1 / s0.clamp(min=1)
            bbar = sb / s0.clamp(min=1)
            sdd = s2 - s1 * dbar
            slope = torch.where(sdd > 1e-6, (sdb - s1 * bbar) / sdd.clamp(min=1e-6), 0.0)
            st = today - (bbar - slope * dbar)
            out[:, f] = torch.where((s0 > 0) & torch.isfinite(today), st, float("nan"))
        return out

    def calibrate_level(self, rows: Optional[torch.Tensor] = None) -> None:
        """Spread of the level statistic per (series, feature): the RMS of the
        statistic at ``level_cal`` offsets over the last day (each with at least
        one earlier day behind it), floored at 1e-6 of the series' std."""
        geo = self._level_geometry()
        if geo is None:
            self.lvl_sig = None
            return
        newest, avail, K, step = geo
        if self.gpu:
            from ..ops import lstm as L
            st = L.lstm_level([r.data for r in self.rings], newest, avail, self.season, self.level_points,
                              K=K, back_step=step)
        else:
            st = torch.stack([self._level_stat_cpu((k + 1) * step) for k in range(K)])
        ok = torch.isfinite(st)
        cnt = ok.sum(0)
        ms = torch.where(ok, st * st, 0.0).sum(0) / cnt.clamp(min=1)
        sig = ms.sqrt().clamp(min=1e-12)
        sig = torch.maximum(sig, self.std * 1e-6)
        sig = torch.where(cnt >= 4, sig, torch.full_like(sig, float("inf")))  # too little history: no level term
        if rows is None or self.lvl_sig is None:
            full = torch.full((self.n, self.F), float("inf"), device=self.device)
            sel = self._all if rows is None else rows.to(self.device, torch.long)
            full[sel] = sig[sel]
            self.lvl_sig = full.contiguous()
        else:
            sel = rows.to(self.device, torch.long)
            self.lvl_sig[sel] = sig[sel]

    def level_z(self, head_dev: bool = False) -> Optional[torch.Tensor]:
        """``[n, F]`` level z of every series' newest points (None: no level term);
        ``head_dev``: the newest column relative to the graph record's device head."""
        if self.lvl_sig is None or self.level_threshold is None:
            return None
        r0 = self.rings[0]
        if r0.length < self.level_points + self.LVL_E + self.season:
            return None
        if self.gpu:
            from ..ops import lstm as L
            newest = r0.length - 1 if head_dev else (r0.head + r0.length - 1) % r0.R
            self._zl = L.lstm_level([r.data for r in self.rings], newest, r0.length, self.season,
                                    self.level_points, sig=self.lvl_sig, out=self._zl,
                                    head_dev=self._grec_dev[1:2] if head_dev else None)
            return self._zl
        st = self._level_stat_cpu(0)
        return torch.where(torch.isfinite(st) & (self.lvl_sig > 0), st / self.lvl_sig, 0.0)

    def _calib_errors(self, src, n: int) -> torch.Tensor:
        """Reconstruction errors (float64) of ``src``'s windows: a kernel
        ``RingSource`` on the GPU, a ``[B, T, F]`` window tensor on the CPU
        (``None``: ``n`` random history windows)."""
        if self.gpu:
            from ..ops import lstm as L
            self._pack_scoring()
            return L.lstm_score(self.packed, None, 0.0, 1.0, thr_default=float("inf"), ring=src,
                                T=self.T)["err"].double()
        with torch.no_grad():
            return self.model.recon_error(self._sample(n) if src is None else src).double()

    @staticmethod
    def _all_reduce(t: torch.Tensor) -> None:
        if comm.active():
            dist.all_reduce(t)

    def _pack_scoring(self) -> None:
        from ..ops import lstm as L
        if self.packed is None:
            self.packed = L.pack(self.model, fp8=self.fp8, device=self.device)
        else:
            L.repack_into(self.packed, self.model)

    def _level_args(self, ring) -> Optional[Dict]:
        """The scoring kernel's fused level term (None: no level term yet)."""
        if self.lvl_sig is None or self.level_threshold is None:
            return None
        r0 = self.rings[0]
        if r0.length < self.level_points + self.LVL_E + self.season:
            return None
        newest = r0.length - 1 if ring.head_dev is not None else (r0.head + r0.length - 1) % r0.R
        return {"sig": self.lvl_sig, "m": self.season, "E": self.LVL_E, "newest": newest, "avail": r0.length}

    def _score_packed(self, zeroed: bool = False, ring=None) -> Dict[str, torch.Tensor]:
        """The fused scoring kernel, the level term computed inside it; ``zeroed``: the
        caller has already zeroed the per-app counters on this stream."""
        from ..ops import lstm as L
        if not zeroed:
            self.app_stats.zero_()
        ring = ring if ring is not None else self._ring_src()
        self.out = L.lstm_score(self.packed, None, self.mu, self.sigma, thr_default=self.threshold,
                                app_id=self.app_id, app_stats=self.app_stats, out=self.out,
                                ring=ring, T=self.T, cal=self.cal, cal_ewma=self.cal_ewma,
                                thr_level=float(self.level_threshold or float("inf")), level=self._level_args(ring))
        return self.out

    def tick(self, newx: torch.Tensor, train: bool = True, overlap: bool = True) -> Dict[str, torch.Tensor]:
        """Ingest + (optional) DP training step + scoring of every series.

        On the GPU with ``overlap`` the training step runs on a side HIP stream
        concurrently with scoring (the training kernel occupies B/32 SIMD
        pairs, scoring fills the rest); it is enqueued first so that its waves
        are resident before the scoring grid fills the GPU. The scoring weights
        are repacked on the main stream before the side stream forks, so
        scoring uses the weights from before this tick's update (a one-step
        model lag) and never races the Adam step; the tick joins both streams."""
        if self._graph_ready(train, overlap):
            return self._tick_graph(newx)
        self.ingest_tick(newx)
        if not (train and overlap and self.gpu):
            if train:
                self.train_step()
            return self.score()
        self._pack_scoring()  # before the wait: the side stream's Adam step must not race the repack
        main = torch.cuda.current_stream(self.device)
        self._side_stream().wait_stream(main)
        self.app_stats.zero_()
        if self.fused_train:
            # host order: training kernel, scoring kernel, then the training
            # tail (GEMMs, grad scatter, all-reduce, Adam) whose host cost now
            # overlaps both kernels instead of delaying the scoring launch
            with torch.cuda.stream(self._side):
                self.fg.launch(self.model, None, self._sample_ring(self.train_batch))
            out = self._score_packed(zeroed=True)
            with torch.cuda.stream(self._side):
                self.trainer.step(None, grad_fn=lambda m, _w: self.fg.finish(m))
        else:
            with torch.cuda.stream(self._side):
                self.train_step()
            out = self._score_packed(zeroed=True)
        main.wait_stream(self._side)
        return out

    # ------------------------------------------------------------------ whole-tick HIP graph
    def _graph_ready(self, train: bool, overlap: bool) -> bool:
        """Steady-state training ticks on one GPU run as ONE graph replay: the ring is
        full (the window offsets from the head are constant), this tick does not
        refresh the series statistics, no collective is involved."""
        if not (self.graph_on and train and overlap and self.fused_train):
            return False
        r0 = self.rings[0]
        return (r0.length == r0.R and r0.R > self.T and (self.ticks + 1) % self.restat_every != 0
                and not comm.active())

    def _tick_body(self, newx: torch.Tensor) -> Dict[str, torch.Tensor]:
        """The graph's launches: record step, ring appends at the device column, repacks,
        training windows sampled, counters zeroed, fork; training kernel (side), scoring
        with the fused level term (main), training tail + Adam (side); join."""
        from ..ops import kernels as K
        main = torch.cuda.current_stream(self.device)
        self._grec_dev.add_(1).remainder_(self.rings[0].R)  # the previous tick's positions -> this tick's
        for f, ring in enumerate(self.rings):
            K.ring_append(ring.data, 0, newx[:, f:f + 1], col_dev=self._grec_dev[0:1])
        self._pack_scoring()
        # the training step's sampling and packing before the fork: after it each branch
        # starts with its big kernel, the training kernel created first, so its waves are
        # resident before scoring fills the GPU (in a graph the stream priority does not order
        # the branches; a starved training kernel runs after the scoring grid, not beside it)
        ring_tr = self._sample_ring_dev(self.train_batch)
        self.fg.pack(self.model)
        self.app_stats.zero_()
        side = self._side_stream()
        side.wait_stream(main)
        with torch.cuda.stream(side):
            self.fg.launch(self.model, None, ring_tr, pack=False)
        out = self._score_packed(zeroed=True, ring=self._ring_src_dev())
        with torch.cuda.stream(side):
            self.trainer.step(None, grad_fn=lambda m, _w: self.fg.finish(m))
        main.wait_stream(side)
        return out

    def _tick_graph(self, newx: torch.Tensor) -> Dict[str, torch.Tensor]:
        """One steady-state tick as a HIP-graph replay (captured on the first such tick,
        whose work runs eagerly; re-captured when anything the graph bakes in moved:
        buffers, the calibration constants, the sampled rows).  The host mirrors the
        ring bookkeeping; the replay steps the device record of ring positions itself, so
        the host writes nothing per tick and a caller may enqueue the next tick before
        this one ran.  The record is re-written (as the previous tick's positions) only
        when the rings moved since the last graph tick by anything but one step."""
        r0 = self.rings[0]
        R = r0.R
        col = r0.next_col()
        for ring in self.rings:
            ring.advance(1)
        self.ticks += 1
        now = (col, r0.head)
        last = self._grec_last
        if last is None or ((last[0] + 1) % R, (last[1] + 1) % R) != now:
            rec = self._grec_host[self._grec_k % 4]
            self._grec_k += 1
            rec[0], rec[1] = (col - 1) % R, (r0.head - 1) % R
            self._grec_dev.copy_(rec, non_blocking=True)
        self._grec_last = now
        live = None if self.live is None else (self.live.data_ptr(), self.live.numel())
        key = (newx.data_ptr(), tuple(newx.shape), tuple(r.data.data_ptr() for r in self.rings), live,
               None if self.lvl_sig is None else self.lvl_sig.data_ptr(), self.level_threshold,
               None if self.cal is None else self.cal.data_ptr(), self.cal_ewma, self.mu, self.sigma,
               self.threshold, self.app_stats.data_ptr(), self.app_id.data_ptr(), id(self.packed))
        if self._graph is not None and key == self._graph_key:
            self._graph.replay()
            self.graph_replays += 1
            self.trainer.steps += 1
            return self.out
        out = self._tick_body(newx)            # this tick eagerly (builds every buffer) ...
        torch.cuda.current_stream(self.device).synchronize()
        g = torch.cuda.CUDAGraph()             # ... the next ones as one replay
        g.register_generator_state(self.gen)
        steps = self.trainer.steps
        with torch.cuda.graph(g):
            self._tick_body(newx)
        self.trainer.steps = steps             # the capture ran no step
        self._graph, self._graph_key = g, key
        return out

    def _side_stream(self):
        if self._side is None:
            # high-priority side stream: the long, latency-bound training kernel
            # (B/32 wave pairs) must get its CU slots before the scoring grid
            # (N/32 waves, enough to fill the GPU) takes them all
            self._side = torch.cuda.Stream(self.device, priority=-1)
        return self._side

    def score(self) -> Dict[str, torch.Tensor]:
        if self.gpu:
            self._pack_scoring()
            return self._score_packed()
        x = self._gather(self._all, self._zero_off)
        self.app_stats.zero_()
        with torch.no_grad():
            err = self.model.recon_error(x)
        z = (err - self.mu) / max(self.sigma, 1e-12)
        zs = None
        if self.cal is not None:
            zs = (err - self.cal[:, 0]) * self.cal[:, 1]
            z = torch.minimum(z, zs)
        v = z > self.threshold
        zl = self.level_z()
        if zl is not None:  # same level term as the kernel epilogue
            v = v | (zl.abs().amax(1) > float(self.level_threshold))
        v = v.to(torch.int8)
        if self.cal is not None and self.cal_ewma > 0:  # same update (and gate) as the kernel epilogue
            upd = (v == 0) & torch.isfinite(err) & (zs <= CAL_GATE)
            nmu = self.cal[:, 0] + self.cal_ewma * (err - self.cal[:, 0])
            nmu = torch.where(upd, nmu, self.cal[:, 0])
            self.cal[:, 1] *= self.cal[:, 0] / nmu
            self.cal[:, 0] = nmu
        ids = self.app_id.long()
        self.app_stats.index_put_((ids, torch.zeros_like(ids)), v.int(), accumulate=True)
        self.app_stats.index_put_((ids, torch.ones_like(ids)), torch.ones_like(v, dtype=torch.int32),
                                  accumulate=True)
        self.out = {"err": err, "zscore": z, "verdict": v}
        return self.out
