"""Batched scoring of heterogeneous analysis jobs.

The service-path counterpart of :mod:`foremast_amd.brain.engine`: each
(job, metric alias) becomes a :class:`MetricTask` (historical window on its
own grid, pooled current points with their own timestamps, pooled baseline
values).  Tasks are packed into padded tensors — histories front-padded so
their last samples align, per-series forecast horizons computed from the
timestamps — and scored in one pass per model family with the same gfx950
kernels as the streaming engine (rank tests → model fit with the fused
band/verdict epilogue).  On CPU the PyTorch references run instead.

Model selection per ``ML_ALGORITHM`` (design decision, docs/SCORING.md):
``holt_winters`` needs two full seasons of history, otherwise the task falls
back to ``double_exponential_smoothing``; ``bivariate_normal`` applies to
jobs with >= 2 metrics (first two aliases, sorted), ``lstm`` to jobs with
>= 3 metrics; other jobs fall back to ``moving_average_all``.
"""

from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from ..models import bivariate as biv_ref
from ..models import detect as det_ref
from ..models import moving_average as ma_ref
from ..models import pairwise as pw_ref
from ..models import prophet_lite as pl_ref
from ..models import smoothing as sm_ref
from ..utils.config import BrainConfig


@dataclass
class MetricTask:
    job_id: str
    alias: str
    metric: str
    namespace: str
    app: str
    step: float
    hist: np.ndarray            # [T] float32, NaN gaps, on the historical grid
    hist_end: float             # timestamp of hist[-1]
    cur_ts: np.ndarray          # [C] float64
    cur_vals: np.ndarray        # [C] float32
    cur_tags: List[str] = field(default_factory=list)
    base_vals: Optional[np.ndarray] = None
    threshold: float = 2.0
    bound: int = 1
    min_lower: float = 0.0
    caller: str = ""            # split value: the calling service (downstream) or request path (api)
    base_alias: str = ""        # the job's metric alias (alias = "<base_alias>[<split_label>=<caller>]")
    split_label: str = ""       # "caller" | "uri" | "" (not split)


@dataclass
class TaskResult:
    verdict: int                       # 1 anomalous, 0 healthy, -1 unknown
    anomalies: List[Tuple[float, float, str]]
    upper: np.ndarray
    lower: np.ndarray
    model: str
    p_values: Optional[Tuple[float, float, float]] = None
    differs: bool = False


class BatchScorer:
    def __init__(self, cfg: Optional[BrainConfig] = None, device: Optional[torch.device] = None) -> None:
        self.cfg = cfg or BrainConfig()
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
        self.device = torch.device(device)
        self.gpu = self.device.type == "cuda"
        self.series_scored = 0

    # ------------------------------------------------------------------ packing
    def _season_points(self, step: float) -> int:
        return max(2, int(round(self.cfg.season * 60.0 / step))) if step > 0 else self.cfg.season

    def _pack(self, tasks: List[MetricTask]):
        B = len(tasks)
        T = max(len(t.hist) for t in tasks)
        T = (T + 7) // 8 * 8  # rows 16/32-byte aligned for the kernels' vector loads (front NaN pad)
        C = max(1, max(len(t.cur_vals) for t in tasks))
        hist = np.full((B, T), np.nan, dtype=np.float32)
        cur = np.full((B, C), np.nan, dtype=np.float32)
        hz = np.ones((B, C), dtype=np.int32)
        for i, t in enumerate(tasks):
            if len(t.hist):
                hist[i, T - len(t.hist):] = t.hist
            c = len(t.cur_vals)
            cur[i, :c] = t.cur_vals
            if c:
                h = np.rint((t.cur_ts - t.hist_end) / t.step).astype(np.int64)
                hz[i, :c] = np.clip(h, 1, 1 << 20)
        nb = max([len(t.base_vals) for t in tasks if t.base_vals is not None] + [0])
        base = None
        if nb:
            base = np.full((B, nb), np.nan, dtype=np.float32)
            for i, t in enumerate(tasks):
                if t.base_vals is not None:
                    base[i, :len(t.base_vals)] = t.base_vals
        thr = np.array([t.threshold for t in tasks], dtype=np.float32)
        bnd = np.array([t.bound for t in tasks], dtype=np.int8)
        low = np.array([t.min_lower for t in tasks], dtype=np.float32)
        return hist, cur, hz, base, thr, bnd, low

    # ------------------------------------------------------------------ scoring
    def score(self, tasks: List[MetricTask], algorithm: Optional[str] = None) -> List[TaskResult]:
        algorithm = (algorithm or self.cfg.algorithm).lower()
        results: List[Optional[TaskResult]] = [None] * len(tasks)
        groups: Dict[Tuple[str, int], List[int]] = {}
        for i, t in enumerate(tasks):
            algo = algorithm
            m = self._season_points(t.step)
            if algo == "holt_winters" and np.count_nonzero(~np.isnan(t.hist)) and len(t.hist) < 2 * m:
                algo = "double_exponential_smoothing"
            if algo == "seasonal_decompose" and len(t.hist) < 2 * m + 1:
                algo = "moving_average_all"  # needs more than two seasons of history
            if algo in ("bivariate_normal", "lstm", "auto"):
                algo = "moving_average_all"  # per-metric part; the joint model runs in the worker
            groups.setdefault((algo, m if algo in ("holt_winters", "seasonal_decompose") else 0), []).append(i)
        for (algo, m), idx in groups.items():
            sub = [tasks[i] for i in idx]
            for i, r in zip(idx, self._score_group(sub, algo, m)):
                results[i] = r
        self.series_scored += len(tasks)
        return results  # type: ignore[return-value]

    def _score_group(self, tasks: List[MetricTask], algo: str, m: int) -> List[TaskResult]:
        cfg = self.cfg
        hist, cur, hz, base, thr, bnd, low = self._pack(tasks)
        B = len(tasks)
        dev = self.device
        t_cur = torch.from_numpy(cur).to(dev)
        differs = None
        pvals = None
        bmean = None  # the baseline window means (mean-shift rule)
        if base is not None and cfg.pairwise_algorithm.upper() != "NONE":
            mode = pw_ref.PW_BY_NAME.get(cfg.pairwise_algorithm.upper(), pw_ref.PW_ALL)
            t_base = torch.from_numpy(base).to(dev)
            bmean = torch.nanmean(t_base.float(), 1).contiguous()
            if self.gpu:
                from ..ops import kernels as K
                o = K.rank_tests(t_base, t_cur, mode, cfg.pairwise_threshold, cfg.min_mann_white,
                                 cfg.min_wilcoxon, cfg.min_kruskal, pods=(1, 1), min_friedman=cfg.min_friedman)
                differs, pvals = o["differs"], o["pvals"]
            else:
                res = pw_ref.rank_tests(t_base, t_cur)
                differs = pw_ref.pairwise_differs(res, mode, cfg.pairwise_threshold, cfg.min_mann_white,
                                                  cfg.min_wilcoxon, cfg.min_kruskal,
                                                  cfg.min_friedman).to(torch.uint8)
                pvals = torch.stack([res.p_mw, res.p_wilcoxon, res.p_kruskal], 1)
        has_base = torch.tensor([t.base_vals is not None for t in tasks], device=dev)
        if differs is not None:
            differs = torch.where(has_base, differs, torch.zeros_like(differs)).contiguous()
        t_bnd = torch.from_numpy(bnd).to(dev)
        # per-point thresholds of the full and the lowered band for each task's window
        n_pts = torch.tensor([max(1, len(t.cur_vals)) for t in tasks], dtype=torch.float64)
        thr_f, thr_l = det_ref.effective_thresholds(torch.from_numpy(thr), torch.from_numpy(bnd), n_pts,
                                                    cfg.pairwise_scale, cfg.window_correction)
        t_thr, t_thr_low = thr_f.to(dev).contiguous(), thr_l.to(dev).contiguous()
        dkw = dict(threshold_low=t_thr_low, pw_min_points=cfg.pairwise_min_points,
                   shift_threshold=cfg.pairwise_shift, shift_min_points=cfg.pairwise_shift_min_points, base_mean=bmean)
        t_low = torch.from_numpy(low).to(dev)
        t_hz = torch.from_numpy(hz).to(dev)
        t_hist = torch.from_numpy(hist).to(dev)
        mode = sm_ref.MODE_BY_NAME.get(algo)
        if algo == "prophet":
            # batched additive trend + Fourier seasonality (one [B, P, P] solve; torch on the device)
            C = t_cur.shape[1]
            cts = np.zeros((B, C), dtype=np.float64)
            for i, t in enumerate(tasks):
                n = len(t.cur_ts)
                if n:
                    cts[i, :n] = t.cur_ts
                    cts[i, n:] = t.cur_ts[-1]
                else:
                    cts[i, :] = t.hist_end
            ends = torch.tensor([t.hist_end for t in tasks], dtype=torch.float64, device=dev)
            steps = torch.tensor([t.step for t in tasks], dtype=torch.float64, device=dev)
            fit = pl_ref.fit_prophet(t_hist.float(), ends, steps)
            f = pl_ref.forecast(fit, torch.from_numpy(cts).to(dev))
            d = det_ref.detect(f, fit.sigma.float(), t_cur, t_thr, t_bnd, t_low, differs=differs,
                               pairwise_scale=cfg.pairwise_scale,
                               model_ok=fit.n_valid >= cfg.min_historical_points, **dkw)  # no horizon factor
            upper, lower, verdict, anom = d.upper, d.lower, d.verdict, d.anomaly
        elif self.gpu:
            from ..ops import kernels as K
            spec = K.DetectSpec(horizons=t_hz, threshold=t_thr, bound=t_bnd, min_lower=t_low, cur=t_cur,
                                differs=differs, pw_scale=cfg.pairwise_scale, min_valid=cfg.min_historical_points,
                                max_horizon=int(hz.max()) if hz.size and hz.min() >= 1 else None,
                                horizon_variance=cfg.horizon_variance,
                                shift_one_step=cfg.pairwise_shift_one_step, **dkw)
            T = t_hist.shape[1]
            if algo == "seasonal_decompose":
                out = K.decompose_score(t_hist, 0, T, m, spec)
            elif mode is not None:
                g = sm_ref.make_grid(mode, cfg.hw_alpha, cfg.hw_beta, cfg.hw_gamma).to(dev)
                out = K.smoothing_fit(t_hist, 0, T, mode, m if mode == sm_ref.MODE_HW else 1, g, spec)
            else:
                h = t_hist
                head, length = 0, T
                if algo == "moving_average" and cfg.ma_window < T:
                    head, length = T - cfg.ma_window, cfg.ma_window
                out = K.window_stats(h, head, length, spec)
            upper, lower = out["upper"], out["lower"]
            verdict = out["verdict"]
            anom = None
        else:
            if algo == "seasonal_decompose":
                from ..models import decompose as dec_ref
                fc = dec_ref.decompose_forecast(t_hist, m)
                f = dec_ref.forecast_decomposition(fc, t_hz)
                sigma, n_valid = fc.sigma, fc.n_valid
                sigma1 = sigma
            elif mode is not None:
                grid = sm_ref.make_grid(mode, cfg.hw_alpha, cfg.hw_beta, cfg.hw_gamma)
                fit = sm_ref.fit_smoothing(t_hist, mode, grid, m=max(m, 1))
                f = sm_ref.forecast(fit, t_hz)
                sigma, n_valid = fit.sigma, fit.n_valid
                sigma1 = sigma
                if cfg.horizon_variance:
                    sigma = sigma[:, None] * det_ref.horizon_sigma_factor(grid[fit.best.long()], mode, max(m, 1), t_hz)
            else:
                st = ma_ref.window_stats(t_hist, cfg.ma_window if algo == "moving_average" else None)
                f = st.mean[:, None].expand(B, t_cur.shape[1])
                sigma, n_valid = st.std, st.count
                sigma1 = sigma
            d = det_ref.detect(f, sigma, t_cur, t_thr, t_bnd, t_low, differs=differs,
                               pairwise_scale=cfg.pairwise_scale, model_ok=n_valid >= cfg.min_historical_points,
                               shift_sigma=sigma1 if cfg.pairwise_shift_one_step else None, **dkw)
            upper, lower, verdict, anom = d.upper, d.lower, d.verdict, d.anomaly
        upper_np = upper.float().cpu().numpy()
        lower_np = lower.float().cpu().numpy()
        verdict_np = verdict.cpu().numpy()
        cur_np = cur
        p_np = pvals.float().cpu().numpy() if pvals is not None else None
        diff_np = differs.cpu().numpy() if differs is not None else None
        out_res = []
        for i, t in enumerate(tasks):
            c = len(t.cur_vals)
            up, lo = upper_np[i, :c], lower_np[i, :c]
            x = cur_np[i, :c]
            valid = ~np.isnan(x)
            b = int(t.bound)
            flags = valid & ((((b & 1) != 0) & (x > up)) | (((b & 2) != 0) & (x < lo)))
            if verdict_np[i] < 0:
                flags[:] = False
            anomalies = [(float(t.cur_ts[j]), float(x[j]), t.cur_tags[j] if j < len(t.cur_tags) else "")
                         for j in np.nonzero(flags)[0]]
            out_res.append(TaskResult(
                verdict=int(verdict_np[i]), anomalies=anomalies, upper=up.copy(), lower=lo.copy(), model=algo,
                p_values=tuple(float(v) for v in p_np[i]) if p_np is not None and t.base_vals is not None else None,
                differs=bool(diff_np[i]) if diff_np is not None else False))
        return out_res

    # ------------------------------------------------------------------ multivariate
    def score_bivariate(self, pairs: List[Tuple[MetricTask, MetricTask]]) -> List[Tuple[int, List[Tuple[float, float]]]]:
        """Score metric pairs of one job each: the current points of each metric are
        averaged across pods per timestamp and restricted to the timestamps both have
        (:func:`~.multivariate.align_job`).  Returns per pair (verdict, anomalous
        points as (timestamp, first metric's value))."""
        from .multivariate import align_job
        if not pairs:
            return []
        B = len(pairs)
        T = max(max(len(a.hist), len(b.hist)) for a, b in pairs)
        hx = np.full((B, T), np.nan, dtype=np.float32)
        hy = np.full((B, T), np.nan, dtype=np.float32)
        aligned = []
        C = 1
        for i, (a, b) in enumerate(pairs):
            hx[i, T - len(a.hist):] = a.hist
            hy[i, T - len(b.hist):] = b.hist
            _h, cts, cur2 = align_job([a, b])
            aligned.append((cts, cur2))
            C = max(C, len(cts))
        cur = np.full((B, C, 2), np.nan, dtype=np.float32)
        for i, (cts, cur2) in enumerate(aligned):
            cur[i, :len(cts)] = cur2
        thr = torch.tensor([a.threshold for a, _ in pairs], dtype=torch.float32, device=self.device)
        if self.gpu:
            from ..ops import kernels as K
            out = K.bivariate(torch.from_numpy(hx).to(self.device), torch.from_numpy(hy).to(self.device), 0, T,
                              torch.from_numpy(cur).to(self.device), thr,
                              min_valid=self.cfg.min_historical_points)
            d2 = out["d2"].cpu().numpy()
            verdict = out["verdict"].cpu().numpy()
        else:
            fit = biv_ref.fit_bivariate(torch.from_numpy(np.stack([hx, hy], 2)))
            d2t = biv_ref.mahalanobis2(fit, torch.from_numpy(cur))
            d2 = d2t.numpy()
            ok = fit.count.numpy() >= self.cfg.min_historical_points
            an = (d2 > (thr.cpu().numpy() ** 2)[:, None]) & ok[:, None]
            verdict = np.where(an.any(1), 1, np.where((~np.isnan(d2)).any(1) & ok, 0, -1))
        res = []
        t2 = (thr.cpu().numpy() ** 2)
        for i, (cts, cur2) in enumerate(aligned):
            pts = [(float(cts[j]), float(cur2[j, 0])) for j in range(len(cts)) if d2[i, j] > t2[i]]
            res.append((int(verdict[i]) if not pts else 1, pts))
        self.series_scored += 2 * B
        return res
