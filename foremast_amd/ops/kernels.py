"""PyTorch-facing launchers for the gfx950 kernels.

Every launcher validates shapes, dtypes, strides and devices on the host
*before* launching (a bad shape must never reach a kernel), allocates any
output not supplied in ``out`` and launches on the current HIP stream.  No
host synchronisation happens here, so the launchers can be captured into a
HIP graph.
"""

from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass
from typing import Tuple, Dict, Optional

import torch

from . import _native as nat

MODE_ES, MODE_DES, MODE_HW = 0, 1, 2
DEFAULT_ES_K = 16  # steps per lane per segment for ES/DES (segment = 1024)
LDS_LIMIT = 64 * 1024          # budget of the tiled kernels (keeps >= 2 workgroups per CU)
D_LDS_LIMIT = 78 * 1024        # HW variant 5: two 4-wave workgroups per CU within 160 KiB
LDS_MAX_WG = 160 * 1024        # gfx950: one workgroup may own the whole 160 KiB


class KernelShapeError(ValueError):
    pass


def _need(cond: bool, msg: str) -> None:
    if not cond:
        raise KernelShapeError(msg)


def _cuda(t: torch.Tensor, name: str) -> None:
    _need(t.is_cuda, f"{name} must be a GPU tensor")


def _vec(t: Optional[torch.Tensor], n: int, dtype, name: str, device) -> Optional[torch.Tensor]:
    if t is None:
        return None
    _need(t.dim() == 1 and t.shape[0] == n, f"{name} must be [{n}], got {tuple(t.shape)}")
    _need(t.dtype == dtype, f"{name} must be {dtype}, got {t.dtype}")
    _need(t.is_contiguous(), f"{name} must be contiguous")
    _need(t.device == device, f"{name} on {t.device}, expected {device}")
    return t


@dataclass
class DetectSpec:
    """Inputs of the fused detection epilogue (see models/detect.py)."""

    horizons: torch.Tensor                 # int32 [C] (shared) or [N, C] (per series)
    threshold: torch.Tensor                # float32 [N]
    bound: torch.Tensor                    # int8 [N]
    min_lower: torch.Tensor                # float32 [N]
    cur: Optional[torch.Tensor] = None     # float32 [N, C] (row stride free)
    differs: Optional[torch.Tensor] = None  # uint8 [N]
    pw_scale: float = 0.5
    min_valid: int = 0
    want_band: bool = True
    app_id: Optional[torch.Tensor] = None   # int32 [N]
    app_stats: Optional[torch.Tensor] = None  # int32 [A, 2]
    anomalies: Optional["AnomalyBuffer"] = None  # K9 compaction of anomalous points
    # host-known upper bound of ``horizons`` (all values in 1..max_horizon); lets the
    # Holt-Winters kernel keep only the seasonal phases the forecast needs (variant 4)
    max_horizon: Optional[int] = None
    # lowered (pairwise) threshold per series (models/detect.py effective_thresholds);
    # None: threshold * pw_scale.  The lowered band needs >= pw_min_points points.
    threshold_low: Optional[torch.Tensor] = None
    pw_min_points: int = 1
    # scale sigma by the h-step forecast-error factor of the fitted smoothing model
    horizon_variance: bool = True
    # > 0: mean-shift rule when ``differs`` (models/detect.py ``shift_threshold``), against
    # ``base_mean`` (float32 [N], the baseline pods' window mean: rank_tests out["base_mean"])
    shift_threshold: float = 0.0
    base_mean: Optional[torch.Tensor] = None
    shift_min_points: int = 1
    # the mean-shift rule's spread: the one-step sigma (models/detect.py ``shift_sigma``)
    # instead of the horizon-scaled band sigma
    shift_one_step: bool = False
    # window-corrected thresholds tabulated by (class, valid points) (detect.h det_thresholds):
    # float32 [classes, 2, n] and uint16-in-int16 [N] classes; replaces threshold / threshold_low
    thr_lut: Optional[torch.Tensor] = None
    thr_cls: Optional[torch.Tensor] = None
    # per-series host record [N, 4] (verdict, valid points, upper / lower at the newest column
    # clamp(tick_min[0] - start_min[n], 0, last_ncol - 1))
    row_out: Optional[torch.Tensor] = None
    start_min: Optional[torch.Tensor] = None
    tick_min: Optional[torch.Tensor] = None
    last_ncol: int = 0


class AnomalyBuffer:
    """Device-side compacted list of anomalous points (K9): the detection
    epilogue appends ``(series, column, value)`` triples; the host copies back
    only ``count`` and the used prefix instead of whole ``[N, C]`` bands."""

    def __init__(self, cap: int, device, count: Optional[torch.Tensor] = None) -> None:
        """``count``: an int32 [1] device tensor to count in (e.g. the tail of a
        per-tick record copied back in one piece); default: its own."""
        dev = torch.device(device)
        self.cap = int(cap)
        self.count = torch.zeros(1, dtype=torch.int32, device=dev) if count is None else count
        dev = self.count.device  # "cuda" -> "cuda:<current>"
        _need(self.count.dtype == torch.int32 and self.count.numel() == 1 and self.count.is_cuda,
              "count must be an int32 [1] GPU tensor")
        self.series = torch.empty(self.cap, dtype=torch.int32, device=dev)
        self.col = torch.empty(self.cap, dtype=torch.int32, device=dev)
        self.val = torch.empty(self.cap, dtype=torch.float32, device=dev)

    def reset(self) -> None:
        self.count.zero_()

    def fetch(self, n_all: Optional[int] = None):
        """(series, col, val) numpy arrays sorted by (series, col), and whether
        the buffer overflowed (more anomalies than ``cap``).  ``n_all``: the count
        when the caller already copied it back."""
        import numpy as np
        if n_all is None:
            n_all = int(self.count.item())
        n = min(n_all, self.cap)
        if n == 0:
            z = np.zeros(0, dtype=np.int32)
            return z, z, np.zeros(0, dtype=np.float32), False
        s = self.series[:n].cpu().numpy()
        c = self.col[:n].cpu().numpy()
        v = self.val[:n].cpu().numpy()
        order = np.lexsort((c, s))
        return s[order], c[order], v[order], n_all > self.cap


def _fill_detect(d: nat.DetectArgs, spec: DetectSpec, N: int, device, out: Dict[str, torch.Tensor]) -> None:
    hz = spec.horizons
    _need(hz.dtype == torch.int32 and hz.stride(-1) == 1 and hz.dim() in (1, 2),
          "horizons must be int32 [C] or [N, C] with unit inner stride")
    C = int(hz.shape[-1])
    if hz.dim() == 2:
        _need(hz.shape[0] == N, f"per-series horizons must be [{N}, C]")
    _need(spec.horizons.device == device, "horizons on wrong device")
    _vec(spec.threshold, N, torch.float32, "threshold", device)
    _vec(spec.bound, N, torch.int8, "bound", device)
    _vec(spec.min_lower, N, torch.float32, "min_lower", device)
    _vec(spec.differs, N, torch.uint8, "differs", device)
    _vec(spec.threshold_low, N, torch.float32, "threshold_low", device)
    if spec.cur is not None:
        c = spec.cur
        _need(c.dim() == 2 and c.shape[0] == N and c.shape[1] == C,
              f"cur must be [{N}, {C}], got {tuple(c.shape)}")
        _need(c.dtype == torch.float32 and c.stride(1) == 1, "cur must be float32 with unit inner stride")
        _need(c.device == device, "cur on wrong device")
    if spec.app_id is not None:
        _vec(spec.app_id, N, torch.int32, "app_id", device)
        _need(spec.app_stats is not None and spec.app_stats.dtype == torch.int32
              and spec.app_stats.is_contiguous() and spec.app_stats.dim() == 2
              and spec.app_stats.shape[1] == 2, "app_stats must be contiguous int32 [A, 2]")
    kw = dict(dtype=torch.float32, device=device)
    if spec.want_band and C > 0:
        for k in ("forecast", "upper", "lower"):
            if k not in out:
                out[k] = torch.empty((N, C), **kw)
    if "count" not in out:
        out["count"] = torch.empty(N, dtype=torch.int32, device=device)
    if "verdict" not in out:
        out["verdict"] = torch.empty(N, dtype=torch.int8, device=device)
    if "score" not in out:
        out["score"] = torch.empty(N, **kw)
    ab = spec.anomalies
    if ab is not None:
        _need(ab.count.device == device, "anomaly buffer on wrong device")
        d.anom_count, d.anom_series, d.anom_col, d.anom_val = (nat.ptr(ab.count), nat.ptr(ab.series),
                                                               nat.ptr(ab.col), nat.ptr(ab.val))
        d.anom_cap = ab.cap
    d.horizons = nat.ptr(spec.horizons)
    d.h_ld = int(hz.stride(0)) if hz.dim() == 2 else 0
    d.C = C
    d.min_valid = int(spec.min_valid)
    d.cur = nat.ptr(spec.cur)
    d.ld_cur = int(spec.cur.stride(0)) if spec.cur is not None else 0
    d.threshold = nat.ptr(spec.threshold)
    d.bound = nat.ptr(spec.bound)
    d.min_lower = nat.ptr(spec.min_lower)
    d.differs = nat.ptr(spec.differs)
    d.pw_scale = float(spec.pw_scale)
    d.pw_min_points = int(spec.pw_min_points)
    d.shift_thr = float(spec.shift_threshold)
    d.base_mean = nat.ptr(spec.base_mean)
    d.shift_min_points = int(spec.shift_min_points)
    d.shift_one_step = int(bool(spec.shift_one_step))
    d.threshold_low = nat.ptr(spec.threshold_low)
    d.hv_grid, d.hv_mode, d.hv_m = None, 0, 0
    d.forecast = nat.ptr(out.get("forecast"))
    d.upper = nat.ptr(out.get("upper"))
    d.lower = nat.ptr(out.get("lower"))
    d.count = nat.ptr(out["count"])
    d.verdict = nat.ptr(out["verdict"])
    d.score = nat.ptr(out["score"])
    d.app_id = nat.ptr(spec.app_id)
    d.app_stats = nat.ptr(spec.app_stats)
    d.thr_lut, d.thr_cls, d.lut_n = None, None, 0
    if spec.thr_lut is not None:
        lut = spec.thr_lut
        _need(lut.dim() == 3 and lut.shape[1] == 2 and lut.dtype == torch.float32 and lut.is_contiguous()
              and lut.device == device and lut.shape[2] >= 1, "thr_lut must be contiguous float32 [K, 2, n]")
        _vec(spec.thr_cls, N, torch.int16, "thr_cls", device)
        d.thr_lut, d.thr_cls, d.lut_n = nat.ptr(lut), nat.ptr(spec.thr_cls), int(lut.shape[2])
    d.row_out, d.start_min, d.tick_min, d.last_ncol = None, None, None, 0
    if spec.row_out is not None:
        ro = spec.row_out
        _need(ro.dim() == 2 and ro.shape == (N, 4) and ro.dtype == torch.float32 and ro.is_contiguous()
              and ro.device == device, f"row_out must be contiguous float32 [{N}, 4]")
        _vec(spec.start_min, N, torch.int32, "start_min", device)
        _need(spec.tick_min is not None and spec.tick_min.dtype == torch.int32 and spec.tick_min.device == device,
              "row_out needs tick_min (int32 device scalar)")
        _need(1 <= spec.last_ncol <= C, "last_ncol must be in 1..C")
        d.row_out, d.start_min, d.tick_min = nat.ptr(ro), nat.ptr(spec.start_min), nat.ptr(spec.tick_min)
        d.last_ncol = int(spec.last_ncol)


def _set_hvar(d: nat.DetectArgs, spec: DetectSpec, grid: torch.Tensor, mode: int, m: int) -> None:
    """h-step forecast-error scaling of sigma from the fitted grid point (detect.h
    ``hstep_factor``); call after :func:`_fill_detect`."""
    if spec.horizon_variance:
        d.hv_grid = nat.ptr(grid)
        d.hv_mode = {MODE_ES: 1, MODE_DES: 2, MODE_HW: 3}[int(mode)]
        d.hv_m = int(m) if mode == MODE_HW else 0


def _hist_check(hist: torch.Tensor, head: int, length: int) -> None:
    _cuda(hist, "hist")
    _need(hist.dim() == 2, "hist must be [N, R]")
    _need(hist.dtype in (torch.float32, torch.bfloat16), "hist must be float32 or bfloat16")
    _need(hist.stride(1) == 1, "hist rows must be contiguous")
    R = hist.shape[1]
    _need(0 <= head < R, f"head {head} out of [0, {R})")
    _need(0 < length <= R, f"length {length} out of (0, {R}]")


UNIFORM_K = (8, 12, 16, 24, 32)
HALF_K = (45, 9)      # variants 4 / 5 (two series per wave): season = 32 * K (variant 4: K = 45 only)
QUAD_K = (18,)        # variant 5, four series per wave (hw_q_kernel): season = 16 * K (288: the 300 s step)
# variant 6 (hw_seq.hip): sequential fit with the season in registers, one (series, grid pair)
# per thread, at the short daily seasons of the 3600 / 1800 / 1200 / 900 / 600 s steps; at the
# 300 s step (m = 288) only with FOREMAST_HW_SEQ288=1 (gap-independent cost: faster than variant 5
# once most series pairs are gapped, slower on dense data)
SEQ_M = (24, 48, 72, 96, 144)
HALF_HB = 16          # seasonal phases kept per series by variant 4 (max forecast horizon)
last_hw_variant: Optional[int] = None  # variant actually launched by the last smoothing_fit (tests/bench)
DEFAULT_HW_VARIANT = 5
last_detect_deferred = False


def smoothing_geometry(mode: int, T: int, m: int, K: Optional[int] = None):
    """Return (Tp, pad, K, seg) for the smoothing kernel.  For Holt-Winters a K
    that divides the season exactly (<= 64 lanes) selects the branch-free
    uniform kernel (1440 = 60 x 24); otherwise K = ceil(m / 64) (guarded)."""
    if mode == MODE_HW:
        _need(m >= 2, "season must be >= 2")
        k = next((c for c in UNIFORM_K if m % c == 0 and m // c <= 64), None) if K is None else K
        if k is None:
            k = (m + 63) // 64
        _need(k <= 32, f"season {m} too long for the register-resident kernel (max 2048)")
        seg = m
        Tp = ((T + m - 1) // m) * m
        _need(Tp // m >= 2, f"holt_winters needs >= 2 seasons (T={T}, m={m})")
    else:
        k = K or DEFAULT_ES_K
        _need(1 <= k <= 32, "K out of range")
        seg = 64 * k
        Tp = ((T + seg - 1) // seg) * seg
    return Tp, Tp - T, k, seg


_PAIR_TAB_CACHE: Dict[tuple, torch.Tensor] = {}


def pair_table(grid: torch.Tensor, K: int) -> torch.Tensor:
    """Per combo-pair precomputed table for the table-driven HW kernel
    (hw_scan.hip ``PairTab``): c1, c2, g1a; pass-1 weights W_i = A^(K-1-i) c;
    B^1, B^2, B^4, B^8, B^16 with B = A^K — all in (forecast, trend)
    coordinates, A = [[1-c1, 1], [-c2, 1]], c = (c1, c2), computed in float64."""
    key = (grid.data_ptr(), tuple(grid.shape), K, grid.device)
    t = _PAIR_TAB_CACHE.get(key)
    if t is not None:
        return t
    import numpy as np
    g = grid.detach().cpu().double().numpy()
    G = g.shape[0]
    npairs = (G + 1) // 2
    size = ((6 + 4 * K + 40) + 15) // 16 * 16
    tab = np.zeros((npairs, size), dtype=np.float64)
    for p in range(npairs):
        for comp, ci in enumerate((2 * p, 2 * p + 1 if 2 * p + 1 < G else 2 * p)):
            al, be, ga = g[ci]
            c2 = al * be
            c1 = al + c2
            A = np.array([[1 - c1, 1.0], [-c2, 1.0]])
            c = np.array([c1, c2])
            tab[p, 0 + comp] = c1
            tab[p, 2 + comp] = c2
            tab[p, 4 + comp] = ga * (1 - al)
            Ap = np.eye(2)
            pows = [np.eye(2)]
            for _ in range(K):
                Ap = A @ Ap
                pows.append(Ap)
            for i in range(K):
                Wi = pows[K - 1 - i] @ c
                tab[p, 6 + 4 * i + comp] = Wi[0]
                tab[p, 6 + 4 * i + 2 + comp] = Wi[1]
            B = pows[K]
            Bp = B
            for r in range(5):
                base = 6 + 4 * K + 8 * r
                for q, v in enumerate((Bp[0, 0], Bp[0, 1], Bp[1, 0], Bp[1, 1])):
                    tab[p, base + 2 * q + comp] = v
                Bp = Bp @ Bp
    # then A^0 .. A^K per pair ([npairs][K + 1][8], Mat2 of v2f: m11, m12, m21, m22 with the
    # two combos interleaved): the gapped-series kernel (hw_dg_kernel) assembles a lane's
    # season map from them run by run
    pw = np.zeros((npairs, K + 1, 8), dtype=np.float64)
    for p in range(npairs):
        for comp, ci in enumerate((2 * p, 2 * p + 1 if 2 * p + 1 < G else 2 * p)):
            al, be, ga = g[ci]
            c2 = al * be
            c1 = al + c2
            A = np.array([[1 - c1, 1.0], [-c2, 1.0]])
            Ap = np.eye(2)
            for n in range(K + 1):
                for q, v in enumerate((Ap[0, 0], Ap[0, 1], Ap[1, 0], Ap[1, 1])):
                    pw[p, n, 2 * q + comp] = v
                Ap = A @ Ap
    t = torch.tensor(np.concatenate([tab.reshape(-1), pw.reshape(-1)]), dtype=torch.float32,
                     device=grid.device).contiguous()
    if len(_PAIR_TAB_CACHE) > 64:
        _PAIR_TAB_CACHE.clear()
    _PAIR_TAB_CACHE[key] = t
    return t


def smoothing_supported(mode: int, T: int, m: int, bf16: bool) -> bool:
    try:
        Tp, _, k, seg = smoothing_geometry(mode, T, m)
    except KernelShapeError:
        return False
    lib = nat.load()
    if lib is None:
        return False
    return lib.fm_smooth_lds_bytes(Tp, m if mode == MODE_HW else 1, seg, int(bf16)) <= LDS_LIMIT


def smoothing_fit(hist: torch.Tensor, head: int, length: int, mode: int, m: int,
                  grid: torch.Tensor, det: DetectSpec, K: Optional[int] = None,
                  want_season: bool = False, out: Optional[Dict[str, torch.Tensor]] = None,
                  variant: Optional[int] = None, head_dev: Optional[torch.Tensor] = None,
                  defer_detect: bool = False, detect_after=None) -> Dict[str, torch.Tensor]:
    """``head_dev`` (int32 device scalar): the ring head is read from device memory
    at run time (HIP-graph replays); only the two-series-per-wave HW variants
    (4/5) support it — other paths raise.

    ``defer_detect``: on the variant 4/5 path the fit skips the band/verdict
    epilogue and stores what it needs (``season_hb``, ``nvalid``); call
    :func:`hw_detect_deferred` afterwards (``det.differs`` is read only then, so
    the rank tests can run concurrently with the fit).  ``last_detect_deferred``
    says whether the request was honoured; when it is not, the fit detects inline
    and, if ``detect_after`` (a stream producing ``det.differs``) is given, the
    current stream first waits for it."""
    global last_detect_deferred
    last_detect_deferred = False
    lib = nat.require()
    _hist_check(hist, head, length)
    dev = hist.device
    N = hist.shape[0]
    _need(grid.dim() == 2 and grid.shape[1] == 3 and grid.dtype == torch.float32
          and grid.is_contiguous() and grid.device == dev, "grid must be contiguous float32 [G, 3] on device")
    G = grid.shape[0]
    _need(G >= 1, "empty grid")
    mm = m if mode == MODE_HW else 1
    Tp, pad, k, seg = smoothing_geometry(mode, length, mm, K)
    bf16 = hist.dtype == torch.bfloat16
    if variant is None:
        variant = int(os.environ.get("FOREMAST_HW_VARIANT", str(DEFAULT_HW_VARIANT)))
    if mode in (MODE_ES, MODE_DES) and variant in (4, 5) and K is None and G <= 64:
        return _es_seq_fit(lib, hist, head, length, mode, grid, det, out, head_dev=head_dev, defer=defer_detect)
    if (mode == MODE_HW and variant in (4, 5) and K is None and G <= 64
            and (mm in SEQ_M or (mm == 288 and os.environ.get("FOREMAST_HW_SEQ288", "0") == "1"))
            and os.environ.get("FOREMAST_HW_SEQ", "1") != "0"
            and (det.horizons.shape[-1] == 0 or (det.max_horizon is not None and 1 <= det.max_horizon <= HALF_HB))
            and lib.fm_hw_seq_lds_bytes(Tp, mm, G) <= LDS_LIMIT):
        return _hw_seq_fit(lib, hist, head, length, mm, grid, det, Tp, pad, out, want_season,
                           head_dev=head_dev, defer=defer_detect, detect_after=detect_after)
    if variant in (4, 5):
        hmax = det.max_horizon
        if (variant == 5 and mode == MODE_HW and bf16 and mm % 16 == 0 and mm // 16 in QUAD_K
                and not want_season and K is None and hmax is not None and 1 <= hmax <= min(mm // 16, HALF_HB)
                and os.environ.get("FOREMAST_HW_QUAD", "1") != "0"
                and lib.fm_hw_q_lds_bytes(Tp, mm, mm // 16) <= D_LDS_LIMIT):
            return _hw_half_fit(lib, hist, head, length, mm, grid, det, Tp, pad, hmax, out, residual=True,
                                head_dev=head_dev, defer=defer_detect, quad=True)
        if (mode == MODE_HW and bf16 and mm % 32 == 0 and mm // 32 in HALF_K and not want_season
                and hmax is not None and 1 <= hmax <= min(mm // 32, HALF_HB) and K is None):
            if variant == 5 and lib.fm_hw_d_lds_bytes(Tp, mm, mm // 32) <= D_LDS_LIMIT:
                return _hw_half_fit(lib, hist, head, length, mm, grid, det, Tp, pad, hmax, out, residual=True,
                                    head_dev=head_dev, defer=defer_detect)
            if mm // 32 == 45 and lib.fm_hw_half_lds_bytes(Tp, mm, mm // 32) <= LDS_LIMIT:
                return _hw_half_fit(lib, hist, head, length, mm, grid, det, Tp, pad, hmax, out, head_dev=head_dev,
                                    defer=defer_detect)
        variant = 3
    if detect_after is not None:
        torch.cuda.current_stream(dev).wait_stream(detect_after)
    _need(head_dev is None, "head_dev needs HW variant 4/5 geometry")
    fast_lds = lib.fm_hw_scan_lds_bytes(Tp, seg, k, int(mode), int(bf16))
    if variant >= 0 and not (seg % k == 0 and seg // k <= 64 and fast_lds <= LDS_LIMIT):
        variant = -1
    global last_hw_variant
    last_hw_variant = variant
    if variant < 0:
        if mode == MODE_HW and k not in (8, 16, 24, 32):
            k = (mm + 63) // 64
        lds = lib.fm_smooth_lds_bytes(Tp, mm, seg, int(bf16))
        _need(lds <= LDS_LIMIT, f"series too long for LDS staging ({lds} bytes)")
    out = {} if out is None else out
    f32 = dict(dtype=torch.float32, device=dev)
    for kname in ("level", "trend", "sigma"):
        if kname not in out:
            out[kname] = torch.empty(N, **f32)
    if "best" not in out:
        out["best"] = torch.empty(N, dtype=torch.int32, device=dev)
    if want_season and mode == MODE_HW and "season" not in out:
        out["season"] = torch.empty((N, mm), **f32)
    a = nat.SmoothArgs()
    a.hist = nat.ptr(hist)
    a.ld = hist.stride(0)
    a.ring_len = hist.shape[1]
    a.head = int(head)
    a.T = int(length)
    a.Tp = Tp
    a.pad = pad
    a.m = mm
    a.K = k
    a.seg = seg
    a.grid = nat.ptr(grid)
    a.G = G
    a.N = N
    a.level = nat.ptr(out["level"])
    a.trend = nat.ptr(out["trend"])
    a.sigma = nat.ptr(out["sigma"])
    a.best = nat.ptr(out["best"])
    a.season_out = nat.ptr(out.get("season")) if (want_season and mode == MODE_HW) else 0
    a.pair_tab = nat.ptr(pair_table(grid, k)) if variant == 3 else 0
    _fill_detect(a.det, det, N, dev, out)
    _set_hvar(a.det, det, grid, mode, mm)
    nat.check(lib.fm_smooth_fit(a, int(mode), int(bf16), int(variant), nat.stream_handle(dev)), "fm_smooth_fit")
    return out


_HALF_WS: Dict[tuple, torch.Tensor] = {}


def _half_workspace(dev, N: int) -> torch.Tensor:
    """Deferred-pair list of variants 4/5 (count, pair starts, done counter),
    reused across calls so a captured tick allocates nothing; allocated zeroed and
    left zeroed by the general kernel (no per-call memset).  One workspace per
    (device, N, stream): fits on two streams never share a count; the kernels
    bound every append by the pair list and the caller zeroes the workspace when a
    launch on this path fails (``_hw_half_fit``)."""
    # inside a HIP-graph capture the workspace must already exist: allocated there it would
    # come from the graph's pool with its zero-fill captured, i.e. re-zeroed at every replay
    # (the gap flags and the deferred-pair total would never survive a tick).  A captured fit
    # uses the (device, N) "graph" workspace that reserve_graph_workspace made beforehand.
    capturing = dev.type == "cuda" and torch.cuda.is_current_stream_capturing()
    key = (dev.index, N, "graph") if capturing else (dev.index, N, nat.stream_handle(dev))
    ws = _HALF_WS.get(key)
    if ws is None and capturing:
        raise RuntimeError("HW workspace allocated inside a graph capture: call reserve_graph_workspace first")
    if ws is None:
        # {count, pairs..., done, total, queue, gap flags...}: total = pairs deferred to the
        # gapped-series kernel since allocation (hw_dg_kernel adds each launch's count); queue =
        # its pair queue; a pair's gap flag sends it straight to that kernel in the next fit
        P = (N + 1) // 2
        ws = torch.zeros(4 + 2 * P, dtype=torch.int32, device=dev)
        _HALF_WS[key] = ws
    return ws


def reserve_graph_workspace(dev, N: int) -> None:
    """Allocate the deferred-pair workspace a captured Holt-Winters fit of N series uses
    (outside the capture; see :func:`_half_workspace`)."""
    dev = torch.device(dev)
    key = (dev.index, N, "graph")
    if key not in _HALF_WS:
        _HALF_WS[key] = torch.zeros(4 + 2 * ((N + 1) // 2), dtype=torch.int32, device=dev)


def hw_deferred_total(dev=None) -> int:
    """Series pairs the variant-5 fit has handed to the gapped-series kernel since the
    workspaces were allocated, over every workspace of ``dev`` (one device sync)."""
    tot = 0
    for (di, _n, _s), ws in _HALF_WS.items():
        if dev is None or di == torch.device(dev).index:
            tot += int(ws[(ws.numel() - 4) // 2 + 2].item())
    return tot


def hw_clear_gap_flags() -> None:
    """Forget which series pairs the last fits found gapped (each is re-staged by the dense
    kernel and re-classified); tests that reuse a shard size with new data call this."""
    for ws in _HALF_WS.values():
        P = (ws.numel() - 4) // 2
        ws[P + 4:].zero_()


SPLIT_MAX = 4096       # HW variant 5 split tail: at most this many series pairs split in two halves
_SPLIT_WS: Dict[int, tuple] = {}


def _split_workspace(dev) -> tuple:
    """Split-tail workspace of variant 5 (hw_scan.hip ``fm_hw_d_fit_split``): int32
    arrival counters [2 * SPLIT_MAX] followed by the halves' candidates (float
    [SPLIT_MAX * 4 * (4 + HALF_HB)]), plus the number of resident workgroup slots
    (two 4-wave workgroups per CU)."""
    hit = _SPLIT_WS.get(dev.index)
    if hit is None:
        words = 2 * SPLIT_MAX + SPLIT_MAX * 4 * (4 + HALF_HB)
        cus = torch.cuda.get_device_properties(dev).multi_processor_count
        hit = (torch.zeros(words, dtype=torch.int32, device=dev), 2 * cus)
        _SPLIT_WS[dev.index] = hit
    return hit


def _hw_half_fit(lib, hist, head, length, m, grid, det, Tp, pad, hmax, out, residual: bool = False,
                 head_dev: Optional[torch.Tensor] = None, defer: bool = False, quad: bool = False):
    """Variants 4/5 of the Holt-Winters fit: two series per wave, season = 32
    lanes x K steps.  Variant 4 (hw_scan.hip ``hw_half_kernel``) walks the
    seasonal state over a bf16 image; variant 5 (``residual``, ``hw_d_kernel``)
    walks D = y - s over an fp32 image of season differences (fewer ops per
    step, at most 7 seasons).  Pairs with gaps past season 0 go to the general
    kernel in both."""
    dev = hist.device
    N = hist.shape[0]
    k = m // 16 if quad else m // 32
    out = {} if out is None else out
    f32 = dict(dtype=torch.float32, device=dev)
    for kname in ("level", "trend", "sigma"):
        if kname not in out:
            out[kname] = torch.empty(N, **f32)
    if "best" not in out:
        out["best"] = torch.empty(N, dtype=torch.int32, device=dev)
    a = nat.SmoothArgs()
    a.hist = nat.ptr(hist)
    a.ld = hist.stride(0)
    a.ring_len = hist.shape[1]
    a.head = int(head)
    a.T = int(length)
    a.Tp = Tp
    a.pad = pad
    a.m = m
    a.K = k
    a.seg = m
    a.grid = nat.ptr(grid)
    a.G = grid.shape[0]
    a.N = N
    a.level = nat.ptr(out["level"])
    a.trend = nat.ptr(out["trend"])
    a.sigma = nat.ptr(out["sigma"])
    a.best = nat.ptr(out["best"])
    a.season_out = 0
    a.pair_tab = nat.ptr(pair_table(grid, k))
    if head_dev is not None:
        _need(head_dev.dtype == torch.int32 and head_dev.device == dev and head_dev.numel() >= 1,
              "head_dev must be an int32 device scalar")
        a.head_dev = nat.ptr(head_dev)
    _fill_detect(a.det, det, N, dev, out)
    _set_hvar(a.det, det, grid, MODE_HW, m)
    if defer:
        for kname, shape in (("season_hb", (N, HALF_HB)), ("nvalid", (N,))):
            if kname not in out:
                out[kname] = torch.empty(shape, **f32)
        a.season_hb = nat.ptr(out["season_hb"])
        a.nvalid_out = nat.ptr(out["nvalid"])
        a.det.C = 0  # no epilogue in the fit
    ws = _half_workspace(dev, N)
    global last_hw_variant, last_detect_deferred
    last_detect_deferred = defer
    if quad:
        # four series per wave at K = m / 16; gapped pairs go to the 32-lane kernel at m / 32
        rc = lib.fm_hw_q_fit(a, nat.ptr(pair_table(grid, m // 32)), int(hmax), nat.ptr(ws), nat.stream_handle(dev))
        if rc != 0:
            ws.zero_()
        nat.check(rc, "fm_hw_q_fit")
        last_hw_variant = 5
        return out
    if residual:
        sws, slots = _split_workspace(dev)
        if os.environ.get("FOREMAST_HW_SPLIT", "1") == "0":
            slots = 0  # whole pairs only
        rc = lib.fm_hw_d_fit_split(a, int(hmax), nat.ptr(ws), nat.ptr(sws), SPLIT_MAX, slots,
                                   nat.stream_handle(dev))
        if rc != 0:
            ws.zero_()  # the general kernel did not run: its self-cleaning reset did not happen
        nat.check(rc, "fm_hw_d_fit_split")
        last_hw_variant = 5
        return out
    rc = lib.fm_hw_half_fit(a, int(hmax), nat.ptr(ws), nat.stream_handle(dev))
    if rc != 0:
        ws.zero_()
    nat.check(rc, "fm_hw_half_fit")
    last_hw_variant = 4
    return out


def _hw_seq_fit(lib, hist, head, length, m, grid, det, Tp, pad, out, want_season: bool,
                head_dev: Optional[torch.Tensor] = None, defer: bool = False, detect_after=None):
    """Variant 6 of the Holt-Winters fit (csrc/hw_seq.hip): short daily seasons (``SEQ_M``),
    one (series, pair of grid points) per thread walking its series from LDS with the m
    seasonal terms in registers; gaps through keep factors on the same path.  The band /
    verdict epilogue is fm_hw_detect_params (inline, or deferred like variants 4 / 5)."""
    dev = hist.device
    N = hist.shape[0]
    out = {} if out is None else out
    f32 = dict(dtype=torch.float32, device=dev)
    for kname in ("level", "trend", "sigma", "nvalid"):
        if kname not in out:
            out[kname] = torch.empty(N, **f32)
    if "best" not in out:
        out["best"] = torch.empty(N, dtype=torch.int32, device=dev)
    if "season_hb" not in out:
        out["season_hb"] = torch.empty((N, HALF_HB), **f32)
    if want_season and "season" not in out:
        out["season"] = torch.empty((N, m), **f32)
    if not defer and detect_after is not None:
        torch.cuda.current_stream(dev).wait_stream(detect_after)  # the inline epilogue reads det.differs
    a = nat.SmoothArgs()
    a.hist = nat.ptr(hist)
    a.ld = hist.stride(0)
    a.ring_len = hist.shape[1]
    a.head = int(head)
    a.T = int(length)
    a.Tp = int(Tp)
    a.pad = int(pad)
    a.m = int(m)
    a.K = 1
    a.seg = int(m)
    a.grid = nat.ptr(grid)
    a.G = grid.shape[0]
    a.N = N
    a.level, a.trend, a.sigma = nat.ptr(out["level"]), nat.ptr(out["trend"]), nat.ptr(out["sigma"])
    a.best = nat.ptr(out["best"])
    a.season_out = nat.ptr(out["season"]) if want_season else 0
    a.nvalid_out = nat.ptr(out["nvalid"])
    a.season_hb = nat.ptr(out["season_hb"])
    if head_dev is not None:
        _need(head_dev.dtype == torch.int32 and head_dev.device == dev and head_dev.numel() >= 1,
              "head_dev must be an int32 device scalar")
        a.head_dev = nat.ptr(head_dev)
    _fill_detect(a.det, det, N, dev, out)
    _set_hvar(a.det, det, grid, MODE_HW, m)
    if defer:
        a.det.C = 0
    global last_hw_variant, last_detect_deferred
    nat.check(lib.fm_hw_seq_fit(a, int(hist.dtype == torch.bfloat16), nat.stream_handle(dev)), "fm_hw_seq_fit")
    last_hw_variant = 6
    last_detect_deferred = defer
    return out


def _es_seq_fit(lib, hist, head, length, mode, grid, det, out, head_dev=None, defer: bool = False):
    """K2 sequential ES / DES grid fit (csrc/es_seq.hip): one thread per series and
    pair of grid points, LDS-staged 64-step chunks; band / verdict by the
    per-series detection kernel (no seasonal term)."""
    _need(head_dev is None, "head_dev needs HW variant 4/5 geometry")
    dev = hist.device
    N = hist.shape[0]
    out = {} if out is None else out
    f32 = dict(dtype=torch.float32, device=dev)
    for kname in ("level", "trend", "sigma", "nvalid"):
        if kname not in out:
            out[kname] = torch.empty(N, **f32)
    if "best" not in out:
        out["best"] = torch.empty(N, dtype=torch.int32, device=dev)
    if "season_hb" not in out:
        out["season_hb"] = torch.zeros((N, HALF_HB), **f32)  # ES / DES forecasts carry no seasonal term
    a = nat.SmoothArgs()
    a.hist = nat.ptr(hist)
    a.ld = hist.stride(0)
    a.ring_len = hist.shape[1]
    a.head = int(head)
    a.T = int(length)
    a.Tp = int(length)
    a.m = 1
    a.K = 1
    a.seg = 1
    a.grid = nat.ptr(grid)
    a.G = grid.shape[0]
    a.N = N
    a.level, a.trend, a.sigma = nat.ptr(out["level"]), nat.ptr(out["trend"]), nat.ptr(out["sigma"])
    a.best = nat.ptr(out["best"])
    a.nvalid_out = nat.ptr(out["nvalid"])
    a.season_hb = nat.ptr(out["season_hb"])
    _fill_detect(a.det, det, N, dev, out)
    _set_hvar(a.det, det, grid, mode, 1)
    if defer:
        a.det.C = 0
    global last_hw_variant, last_detect_deferred
    nat.check(lib.fm_es_seq_fit(a, int(mode), int(hist.dtype == torch.bfloat16), nat.stream_handle(dev)),
              "fm_es_seq_fit")
    last_hw_variant = 5
    last_detect_deferred = defer
    return out


def hw_detect_deferred(out: Dict[str, torch.Tensor], det: DetectSpec, Tp: int, m: int,
                       grid: Optional[torch.Tensor] = None) -> Dict[str, torch.Tensor]:
    """Band / verdict / per-app counters / K9 list for a fit run with
    ``smoothing_fit(..., defer_detect=True)`` (hw_scan.hip ``hw_detect_params_kernel``)."""
    lib = nat.require()
    for kname in ("level", "trend", "sigma", "season_hb", "nvalid"):
        _need(kname in out, f"deferred detection needs out[{kname!r}] from the fit")
    dev = out["level"].device
    N = out["level"].shape[0]
    a = nat.SmoothArgs()
    a.N, a.Tp, a.m = N, int(Tp), int(m)
    a.level, a.trend, a.sigma = nat.ptr(out["level"]), nat.ptr(out["trend"]), nat.ptr(out["sigma"])
    a.season_hb, a.nvalid_out = nat.ptr(out["season_hb"]), nat.ptr(out["nvalid"])
    a.best = nat.ptr(out.get("best"))
    _fill_detect(a.det, det, N, dev, out)
    if grid is not None:
        _need("best" in out, "horizon variance needs out['best'] from the fit")
        _need(grid.dim() == 2 and grid.shape[1] == 3 and grid.dtype == torch.float32 and grid.is_contiguous()
              and grid.device == dev, "grid must be contiguous float32 [G, 3] on device")
        _set_hvar(a.det, det, grid, MODE_HW, m)
    nat.check(lib.fm_hw_detect_params(a, nat.stream_handle(dev)), "fm_hw_detect_params")
    return out


def window_stats(hist: torch.Tensor, head: int, length: int, det: DetectSpec,
                 out: Optional[Dict[str, torch.Tensor]] = None) -> Dict[str, torch.Tensor]:
    lib = nat.require()
    _hist_check(hist, head, length)
    dev = hist.device
    N = hist.shape[0]
    bf16 = hist.dtype == torch.bfloat16
    _need(hist.stride(0) % (8 if bf16 else 4) == 0 and hist.data_ptr() % 16 == 0,
          "hist rows must be 16-byte aligned for vector loads")
    out = {} if out is None else out
    for k in ("mean", "std", "count_hist"):
        if k not in out:
            out[k] = torch.empty(N, dtype=torch.float32, device=dev)
    a = nat.WindowArgs()
    a.hist = nat.ptr(hist)
    a.ld = hist.stride(0)
    a.ring_len = hist.shape[1]
    a.head = int(head)
    a.len = int(length)
    a.N = N
    a.mean = nat.ptr(out["mean"])
    a.stdv = nat.ptr(out["std"])
    a.count = nat.ptr(out["count_hist"])
    _fill_detect(a.det, det, N, dev, out)
    nat.check(lib.fm_window_stats(a, int(bf16), nat.stream_handle(dev)), "fm_window_stats")
    return out


_ZC: Dict[float, float] = {}


def _z_crit(alpha: float) -> float:
    """Two-sided normal quantile isf(alpha / 2) (fp64): p < alpha  <=>  |z| > z_crit."""
    z = _ZC.get(alpha)
    if z is None:
        z = _ZC[alpha] = (float(-torch.special.ndtri(torch.tensor(alpha / 2, dtype=torch.float64)))
                          if 0.0 < alpha < 1.0 else 0.0)
    return z


def rank_tests(base: torch.Tensor, cur: torch.Tensor, mode: int, alpha: float, min_mw: int = 20,
               min_wilcoxon: int = 20, min_kruskal: int = 5, want_pvals: bool = True,
               out: Optional[Dict[str, torch.Tensor]] = None, pods: Optional[Tuple[int, int]] = None,
               min_friedman: int = 5, want_friedman: bool = False) -> Dict[str, torch.Tensor]:
    """K5/K11.  ``pods = (pods_b, pods_c)``: the pod-major window layout the
    Friedman test blocks on (time slot x pod; default one pod per side).  The
    Friedman statistic is computed for mode 6 (FRIEDMAN) or ``want_friedman``
    (``out["friedman"]`` = [N, 2] p-value, complete blocks)."""
    lib = nat.require()
    _cuda(base, "base")
    _need(base.dim() == 2 and cur.dim() == 2 and base.shape[0] == cur.shape[0],
          "base/cur must be [N, nb] / [N, nc]")
    _need(base.dtype == torch.float32 and cur.dtype == torch.float32, "base/cur must be float32")
    _need(base.stride(1) == 1 and cur.stride(1) == 1, "base/cur rows must be contiguous")
    _need(cur.device == base.device, "base/cur on different devices")
    N, nb = base.shape
    nc = cur.shape[1]
    _need(nb >= 1 and nc >= 1, "empty windows")
    _need(lib.fm_rank_lds_bytes(nb, nc) <= LDS_LIMIT, "windows too large for the rank kernel")
    dev = base.device
    out = {} if out is None else out
    if "differs" not in out:
        out["differs"] = torch.empty(N, dtype=torch.uint8, device=dev)
    if "base_mean" not in out:  # the mean-shift rule's centre (DetectSpec.base_mean)
        out["base_mean"] = torch.empty(N, dtype=torch.float32, device=dev)
    if want_pvals:
        if "pvals" not in out:
            out["pvals"] = torch.empty((N, 3), dtype=torch.float32, device=dev)
        if "counts" not in out:
            out["counts"] = torch.empty((N, 3), dtype=torch.float32, device=dev)
    a = nat.RankArgs()
    a.base = nat.ptr(base)
    a.ld_base = base.stride(0)
    a.cur = nat.ptr(cur)
    a.ld_cur = cur.stride(0)
    a.nb, a.nc, a.N, a.mode = nb, nc, N, int(mode)
    a.alpha = float(alpha)
    a.min_mw, a.min_wilcoxon, a.min_kruskal = int(min_mw), int(min_wilcoxon), int(min_kruskal)
    a.pvals = nat.ptr(out.get("pvals")) if want_pvals else 0
    a.counts = nat.ptr(out.get("counts")) if want_pvals else 0
    a.differs = nat.ptr(out["differs"])
    a.base_mean = nat.ptr(out["base_mean"])
    pb, pc = pods if pods is not None else (1, 1)
    fr = want_friedman or int(mode) == 6
    if fr:
        _need(pb >= 1 and pc >= 1 and nb % pb == 0 and nc % pc == 0 and pb + pc <= 64,
              "Friedman needs pod-major windows (nb % pods_b == 0, nc % pods_c == 0, <= 64 pods)")
        if "friedman" not in out:
            out["friedman"] = torch.empty((N, 2), dtype=torch.float32, device=dev)
    a.pods_b, a.pods_c, a.min_friedman = int(pb), int(pc), int(min_friedman)
    a.p_friedman = nat.ptr(out["friedman"]) if fr else 0
    a.z_crit = _z_crit(float(alpha))
    nat.check(lib.fm_rank_tests(a, nat.stream_handle(dev)), "fm_rank_tests")
    return out


def bivariate(hx: torch.Tensor, hy: torch.Tensor, head: int, length: int, cur: torch.Tensor,
              threshold: torch.Tensor, differs: Optional[torch.Tensor] = None, pw_scale: float = 0.5,
              min_valid: int = 0, eps: float = 1e-9, app_id=None, app_stats=None,
              out: Optional[Dict[str, torch.Tensor]] = None) -> Dict[str, torch.Tensor]:
    lib = nat.require()
    _hist_check(hx, head, length)
    _need(hy.shape == hx.shape and hy.dtype == hx.dtype and hy.stride() == hx.stride(),
          "hx/hy must share geometry")
    dev = hx.device
    N = hx.shape[0]
    _need(cur.dim() == 3 and cur.shape[0] == N and cur.shape[2] == 2 and cur.is_contiguous()
          and cur.dtype == torch.float32, "cur must be contiguous float32 [N, C, 2]")
    _vec(threshold, N, torch.float32, "threshold", dev)
    _vec(differs, N, torch.uint8, "differs", dev)
    C = cur.shape[1]
    out = {} if out is None else out
    f32 = dict(dtype=torch.float32, device=dev)
    out.setdefault("mean", torch.empty((N, 2), **f32))
    out.setdefault("cov", torch.empty((N, 3), **f32))
    out.setdefault("d2", torch.empty((N, C), **f32))
    out.setdefault("count", torch.empty(N, dtype=torch.int32, device=dev))
    out.setdefault("verdict", torch.empty(N, dtype=torch.int8, device=dev))
    out.setdefault("score", torch.empty(N, **f32))
    a = nat.BivArgs()
    a.hx, a.hy = nat.ptr(hx), nat.ptr(hy)
    a.ld = hx.stride(0)
    a.ring_len = hx.shape[1]
    a.head, a.len, a.N = int(head), int(length), N
    a.cur = nat.ptr(cur)
    a.C = C
    a.min_valid = int(min_valid)
    a.threshold = nat.ptr(threshold)
    a.differs = nat.ptr(differs)
    a.pw_scale = float(pw_scale)
    a.eps = float(eps)
    for k in ("mean", "cov", "d2", "count", "verdict", "score"):
        setattr(a, k, nat.ptr(out[k]))
    a.app_id = nat.ptr(app_id)
    a.app_stats = nat.ptr(app_stats)
    nat.check(lib.fm_bivariate(a, int(hx.dtype == torch.bfloat16), nat.stream_handle(dev)), "fm_bivariate")
    return out


def ring_append(dst: torch.Tensor, col0: int, src: torch.Tensor, col_dev: Optional[torch.Tensor] = None) -> None:
    """``dst[n, (col0 + j) % R] = src[n, j]`` (dst may be float32 or bf16); ``col_dev``
    (int32 device scalar): added to ``col0`` on the device (graph-captured ticks)."""
    lib = nat.require()
    _cuda(dst, "dst")
    _need(dst.dim() == 2 and src.dim() == 2 and dst.shape[0] == src.shape[0], "shape mismatch")
    _need(dst.stride(1) == 1 and src.stride(1) == 1, "rows must be contiguous")
    _need(src.dtype == torch.float32 and dst.dtype in (torch.float32, torch.bfloat16), "dtype mismatch")
    _need(src.device == dst.device, "device mismatch")
    R = dst.shape[1]
    _need(src.shape[1] <= R, "append wider than the ring")
    if col_dev is not None:
        _need(col_dev.dtype == torch.int32 and col_dev.numel() >= 1 and col_dev.device == dst.device,
              "col_dev must be an int32 device scalar")
    nat.check(lib.fm_ring_append_dev(nat.ptr(dst), dst.stride(0), R, int(col0) % R, nat.ptr(col_dev), src.shape[1],
                                     nat.ptr(src), src.stride(0), dst.shape[0],
                                     int(dst.dtype == torch.bfloat16), nat.stream_handle(dst.device)),
              "fm_ring_append")


DOORBELL_LIMIT = 200_000_000  # wall-clock ticks a doorbell wait spins before giving up (2 s at 100 MHz)


def tick_advance(state: torch.Tensor, R: int, W: int, h_table: Optional[torch.Tensor] = None,
                 h_buf: Optional[torch.Tensor] = None, bell: Optional[torch.Tensor] = None,
                 bell_dev: Optional[torch.Tensor] = None) -> None:
    """Advance the device tick record ``state`` (int32 ``{hist_col, slot,
    graduate, head}``) by one steady-state tick and copy row ``(slot + 1) mod W``
    of ``h_table`` (int32 ``[W, nh]``) into ``h_buf`` (csrc/ingest.hip).
    ``bell`` (pinned host int32 [1]) / ``bell_dev`` (device int32 [2]): first wait until
    the host's counter reaches ``bell_dev[0] + 1`` (the doorbell of a pre-enqueued tick)."""
    lib = nat.require()
    _cuda(state, "state")
    _need(state.dtype == torch.int32 and state.numel() >= 4 and state.is_contiguous(), "state must be int32 [>=4]")
    nh = 0
    if h_table is not None:
        _need(h_buf is not None and h_table.dtype == torch.int32 and h_buf.dtype == torch.int32
              and h_table.dim() == 2 and h_table.shape[0] == W and h_table.is_contiguous() and h_buf.is_contiguous()
              and h_buf.numel() == h_table.shape[1] and h_table.device == state.device
              and h_buf.device == state.device, "h_table must be int32 [W, nh] and h_buf int32 [nh]")
        nh = int(h_table.shape[1])
    if bell is not None:
        _need(bell.dtype == torch.int32 and bell.numel() >= 1 and not bell.is_cuda and bell.is_pinned()
              and bell_dev is not None and bell_dev.dtype == torch.int32 and bell_dev.numel() >= 2
              and bell_dev.device == state.device, "bell must be pinned host int32 [1], bell_dev device int32 [2]")
    nat.check(lib.fm_tick_advance(nat.ptr(state), int(R), int(W), nat.ptr(h_table), nh, nat.ptr(h_buf),
                                  nat.ptr(bell), nat.ptr(bell_dev), DOORBELL_LIMIT if bell is not None else 0,
                                  nat.stream_handle(state.device)), "fm_tick_advance")


def copy_to_host(dst: torch.Tensor, src: torch.Tensor) -> None:
    """Write a small int32 device tensor into a pinned host tensor with a kernel on
    the current stream (system-scope stores; visible to the host after a stream
    sync) instead of a D2H memcpy (csrc/ingest.hip copy_to_host_kernel)."""
    lib = nat.require()
    _cuda(src, "src")
    _need(src.dtype == torch.int32 and src.is_contiguous(), "src must be a contiguous int32 device tensor")
    _need(dst.device.type == "cpu" and dst.is_pinned() and dst.dtype == torch.int32 and dst.is_contiguous()
          and dst.numel() == src.numel(), "dst must be a pinned contiguous int32 host tensor like src")
    nat.check(lib.fm_copy_to_host_i32(dst.data_ptr(), src.data_ptr(), src.numel(), nat.stream_handle(src.device)),
              "fm_copy_to_host_i32")


def tick_ingest(hist: torch.Tensor, hist_col: int, cur: torch.Tensor, P: int, W: int, slot: int,
                newv: torch.Tensor, graduate: bool = True, base: Optional[torch.Tensor] = None,
                newb: Optional[torch.Tensor] = None, state: Optional[torch.Tensor] = None,
                zero: Optional[torch.Tensor] = None) -> None:
    """Per-tick streaming ingest (see csrc/ingest.hip); ``newv``/``newb`` are
    ``[N, P]`` (same row stride) current/baseline pod values.  ``state``: int32
    device ``{hist_col, slot, graduate}`` read at run time instead of the scalar
    arguments (HIP-graph replays; the caller keeps them in range).  ``zero``: a
    contiguous int32 tensor (e.g. the per-app counters) cleared by the same launch."""
    lib = nat.require()
    _cuda(hist, "hist")
    N = hist.shape[0]
    _need(hist.dim() == 2 and hist.stride(1) == 1, "hist must be [N, R] row-contiguous")
    _need(hist.dtype in (torch.float32, torch.bfloat16), "hist dtype")
    _need(cur.dim() == 2 and cur.shape[0] == N and cur.shape[1] == P * W and cur.stride(1) == 1
          and cur.dtype == torch.float32, f"cur must be float32 [N, {P * W}]")
    _need(newv.dim() == 2 and newv.shape[0] == N and newv.shape[1] == P and newv.stride(1) == 1
          and newv.dtype == torch.float32, f"newv must be float32 [N, {P}]")
    # newv / newb may live in pinned host memory: the kernel reads them over the fabric
    # (zero-copy ingest, no separate H2D copy in the tick)
    _need(cur.device == hist.device and (newv.device == hist.device or (newv.device.type == "cpu" and newv.is_pinned())),
          "newv must be on the device or in pinned host memory")
    _need(0 <= slot < W and 0 <= hist_col < hist.shape[1], "slot/hist_col out of range")
    if base is not None:
        _need(newb is not None and base.shape == cur.shape and base.stride() == cur.stride()
              and base.dtype == torch.float32 and base.device == cur.device, "base must match cur")
        _need(newb.shape == newv.shape and newb.stride() == newv.stride() and newb.dtype == torch.float32
              and newb.device == newv.device and (newb.device.type != "cpu" or newb.is_pinned()),
              "newb must match newv")
    nz = 0
    if zero is not None:
        _need(zero.dtype == torch.int32 and zero.is_contiguous() and zero.device == hist.device,
              "zero must be a contiguous int32 tensor on the device")
        nz = int(zero.numel())
    if state is not None:
        _need(state.dtype == torch.int32 and state.device == hist.device and state.numel() >= 3,
              "state must be int32 {hist_col, slot, graduate} on the device")
        nat.check(lib.fm_tick_ingest_dev(nat.ptr(hist), hist.stride(0), nat.ptr(cur), cur.stride(0), int(P), int(W),
                                         nat.ptr(newv), newv.stride(0), N, nat.ptr(base),
                                         nat.ptr(newb) if base is not None else 0,
                                         int(hist.dtype == torch.bfloat16), nat.ptr(state), nat.ptr(zero), nz,
                                         nat.stream_handle(hist.device)), "fm_tick_ingest_dev")
        return
    nat.check(lib.fm_tick_ingest(nat.ptr(hist), hist.stride(0), int(hist_col), nat.ptr(cur), cur.stride(0),
                                 int(P), int(W), int(slot), nat.ptr(newv), newv.stride(0), N, int(graduate),
                                 nat.ptr(base), nat.ptr(newb) if base is not None else 0,
                                 int(hist.dtype == torch.bfloat16), nat.ptr(zero), nz,
                                 nat.stream_handle(hist.device)),
              "fm_tick_ingest")


# ---------------------------------------------------------------------------------
# K4: seasonal decomposition
# ---------------------------------------------------------------------------------

class DecompArgs(C.Structure):
    _fields_ = [("hist", C.c_void_p), ("ld", C.c_longlong), ("ring_len", C.c_int), ("head", C.c_int),
                ("T", C.c_int), ("N", C.c_int), ("m", C.c_int), ("bf16", C.c_int),
                ("trend", C.c_void_p), ("seasonal", C.c_void_p), ("resid", C.c_void_p),
                ("phase_means", C.c_void_p), ("fc_level", C.c_void_p), ("fc_slope", C.c_void_p),
                ("sigma", C.c_void_p), ("nvalid", C.c_void_p), ("det", nat.DetectArgs), ("defer", C.c_void_p),
                ("sfc", C.c_void_p), ("hmax", C.c_int), ("_pad", C.c_int)]


nat.register("fm_seasonal_decompose", [C.POINTER(DecompArgs), C.c_void_p])
nat.register("fm_decompose_lds_bytes", [C.c_int, C.c_int], C.c_size_t)
nat.register("fm_decompose_args_size", [], C.c_longlong)


def seasonal_decompose(hist: torch.Tensor, head: int, length: int, m: int, want=("trend", "seasonal", "resid"),
                       out: Optional[Dict[str, torch.Tensor]] = None) -> Dict[str, torch.Tensor]:
    """Classical additive decomposition of the ring's logical window
    ``[head, head+length)`` (see models/decompose.py); returns float32
    ``trend/seasonal/resid [N, length]`` (those in ``want``) and
    ``phase_means [N, m]``."""
    lib = nat.require()
    _hist_check(hist, head, length)
    _need(2 <= m and 2 * m <= length, f"period {m} needs at least two seasons of history")
    _need(lib.fm_decompose_lds_bytes(length, m) <= LDS_MAX_WG, "window too long for the decomposition kernel")
    N, dev = hist.shape[0], hist.device
    out = {} if out is None else out
    for k in want:
        if k not in out:
            out[k] = torch.empty((N, length), dtype=torch.float32, device=dev)
    if "phase_means" not in out:
        out["phase_means"] = torch.empty((N, m), dtype=torch.float32, device=dev)
    a = DecompArgs()
    a.hist, a.ld, a.ring_len, a.head, a.T, a.N, a.m = nat.ptr(hist), hist.stride(0), hist.shape[1], int(head), \
        int(length), N, int(m)
    a.bf16 = int(hist.dtype == torch.bfloat16)
    a.trend = nat.ptr(out.get("trend"))
    a.seasonal = nat.ptr(out.get("seasonal"))
    a.resid = nat.ptr(out.get("resid"))
    a.phase_means = nat.ptr(out["phase_means"])
    nat.check(lib.fm_seasonal_decompose(C.byref(a), nat.stream_handle(dev)), "fm_seasonal_decompose")
    return out


def decompose_score(hist: torch.Tensor, head: int, length: int, m: int, det: DetectSpec,
                    out: Optional[Dict[str, torch.Tensor]] = None,
                    phase_means: bool = False) -> Dict[str, torch.Tensor]:
    """Seasonal-decomposition scorer (``ML_ALGORITHM=seasonal_decompose``): K4 over
    the ring window without the ``[N, T]`` outputs, forecast = extrapolated trend +
    phase mean, sigma = residual RMS, then the fused band / verdict epilogue
    (models/decompose.py ``decompose_forecast``).  A period with ``m % 16 == 0`` on an
    aligned ring takes the single-pass kernel (gap-free series; a series with a gap
    is finished by the general kernel from a device-side list).  ``phase_means``:
    also write the centred ``[N, m]`` phase means (576 MB at 100k x 1440 — off for
    scoring)."""
    lib = nat.require()
    _hist_check(hist, head, length)
    _need(2 <= m and 2 * m + 1 <= length, f"period {m} needs more than two seasons of history")
    _need(lib.fm_decompose_lds_bytes(length, m) <= LDS_MAX_WG, "window too long for the decomposition kernel")
    N, dev = hist.shape[0], hist.device
    out = {} if out is None else out
    f32 = dict(dtype=torch.float32, device=dev)
    for k in ("level", "slope", "sigma", "nvalid"):
        if k not in out:
            out[k] = torch.empty(N, **f32)
    if phase_means and "phase_means" not in out:
        out["phase_means"] = torch.empty((N, m), **f32)
    if "_defer" not in out or out["_defer"].numel() != N + 2:
        # [count, series..., finished workgroups]: the kernels keep both counts zero between calls
        out["_defer"] = torch.zeros(N + 2, dtype=torch.int32, device=dev)
    a = DecompArgs()
    a.hist, a.ld, a.ring_len, a.head, a.T, a.N, a.m = nat.ptr(hist), hist.stride(0), hist.shape[1], int(head), \
        int(length), N, int(m)
    a.bf16 = int(hist.dtype == torch.bfloat16)
    a.phase_means = nat.ptr(out["phase_means"]) if phase_means else 0
    a.defer = nat.ptr(out["_defer"])
    hmax = det.max_horizon
    if hmax is not None and 1 <= hmax <= 64 and det.horizons is not None:
        # split epilogue: the band / verdict runs in its own kernel from the seasonal terms of
        # horizons 1..hmax (the host-known bound of every horizon)
        if "_sfc" not in out or out["_sfc"].shape != (N, hmax):
            out["_sfc"] = torch.empty((N, hmax), **f32)
        a.sfc, a.hmax = nat.ptr(out["_sfc"]), int(hmax)
    a.fc_level, a.fc_slope = nat.ptr(out["level"]), nat.ptr(out["slope"])
    a.sigma, a.nvalid = nat.ptr(out["sigma"]), nat.ptr(out["nvalid"])
    _fill_detect(a.det, det, N, dev, out)
    nat.check(lib.fm_seasonal_decompose(C.byref(a), nat.stream_handle(dev)), "fm_seasonal_decompose")
    return out


# ---------------------------------------------------------------------------------
# K3 cached model: Holt-Winters state extraction + O(1) update/detect (hw_state.hip)
# ---------------------------------------------------------------------------------

class HwStateArgs(C.Structure):
    _fields_ = [("hist", C.c_void_p), ("ld", C.c_longlong), ("ring_len", C.c_int), ("head", C.c_int),
                ("T", C.c_int), ("Tp", C.c_int), ("m", C.c_int), ("N", C.c_int), ("bf16", C.c_int),
                ("_pad0", C.c_int), ("grid", C.c_void_p), ("best", C.c_void_p), ("level", C.c_void_p),
                ("trend", C.c_void_p), ("season", C.c_void_p), ("nvalid", C.c_void_p)]


class HwUpdateArgs(C.Structure):
    _fields_ = [("hist", C.c_void_p), ("ld", C.c_longlong), ("ring_len", C.c_int), ("col0", C.c_int),
                ("npts", C.c_int), ("t_last", C.c_int), ("m", C.c_int), ("N", C.c_int), ("bf16", C.c_int),
                ("_pad0", C.c_int), ("grid", C.c_void_p), ("best", C.c_void_p), ("level", C.c_void_p),
                ("trend", C.c_void_p), ("season", C.c_void_p), ("sigma", C.c_void_p), ("nvalid", C.c_void_p),
                ("det", nat.DetectArgs)]


nat.register("fm_hw_state", [C.POINTER(HwStateArgs), C.c_void_p])
nat.register("fm_hw_update_detect", [C.POINTER(HwUpdateArgs), C.c_void_p])
nat.register("fm_hw_state_args_size", [], C.c_longlong)
nat.register("fm_hw_update_args_size", [], C.c_longlong)

HW_STATE_MIN_M = 128  # two consecutive 64-step chunks never share a phase (season prefetch)


def hw_state(hist: torch.Tensor, head: int, length: int, m: int, grid: torch.Tensor, best: torch.Tensor,
             state: Optional[Dict[str, torch.Tensor]] = None) -> Dict[str, torch.Tensor]:
    """Full state of the fitted Holt-Winters model at the end of the window
    (models/smoothing.py ``hw_run`` with each series' fitted grid point):
    ``level``/``trend`` ``[N]`` and ``season`` ``[m, N]`` (phase-major, padded-time
    phase), ``nvalid [N]`` (valid points of the fitted steps) and ``Tp`` (padded
    length; the last point has padded time Tp - 1)."""
    lib = nat.require()
    _hist_check(hist, head, length)
    dev, N = hist.device, hist.shape[0]
    _need(m >= HW_STATE_MIN_M, f"cached Holt-Winters needs a season >= {HW_STATE_MIN_M} (got {m})")
    Tp, pad, _, _ = smoothing_geometry(MODE_HW, length, m)
    _need(Tp // m >= 2, "holt_winters needs >= 2 seasons")
    _need(grid.dim() == 2 and grid.shape[1] == 3 and grid.dtype == torch.float32 and grid.is_contiguous()
          and grid.device == dev, "grid must be contiguous float32 [G, 3] on device")
    _vec(best, N, torch.int32, "best", dev)
    state = {} if state is None else state
    f32 = dict(dtype=torch.float32, device=dev)
    for k in ("level", "trend", "nvalid"):
        if k not in state or state[k].shape != (N,):
            state[k] = torch.empty(N, **f32)
    if "season" not in state or state["season"].shape != (m, N):
        state["season"] = torch.empty((m, N), **f32)
    a = HwStateArgs()
    a.hist, a.ld, a.ring_len, a.head = nat.ptr(hist), hist.stride(0), hist.shape[1], int(head)
    a.T, a.Tp, a.m, a.N, a.bf16 = int(length), int(Tp), int(m), N, int(hist.dtype == torch.bfloat16)
    a.grid, a.best = nat.ptr(grid), nat.ptr(best)
    a.level, a.trend, a.season = nat.ptr(state["level"]), nat.ptr(state["trend"]), nat.ptr(state["season"])
    a.nvalid = nat.ptr(state["nvalid"])
    nat.check(lib.fm_hw_state(C.byref(a), nat.stream_handle(dev)), "fm_hw_state")
    state["Tp"] = Tp
    return state


def hw_update_detect(hist: torch.Tensor, col0: int, npts: int, t_last: int, m: int, grid: torch.Tensor,
                     best: torch.Tensor, state: Dict[str, torch.Tensor], sigma: torch.Tensor,
                     nvalid: torch.Tensor, det: DetectSpec,
                     out: Optional[Dict[str, torch.Tensor]] = None) -> Dict[str, torch.Tensor]:
    """Advance the cached state by the ``npts`` points at ring columns ``col0 ..``
    (mod R), the first at padded time ``t_last + 1``, then forecast the current
    window and run the band / verdict epilogue with the refit's ``sigma`` /
    ``nvalid`` / ``best`` (h-step variance of that grid point)."""
    lib = nat.require()
    _cuda(hist, "hist")
    _need(hist.dim() == 2 and hist.stride(1) == 1 and hist.dtype in (torch.float32, torch.bfloat16),
          "hist must be [N, R] row-contiguous float32/bf16")
    dev, N, R = hist.device, hist.shape[0], hist.shape[1]
    _need(0 <= col0 < R and 0 <= npts <= R and t_last >= 0, "col0/npts/t_last out of range")
    _need(state["season"].shape == (m, N) and state["season"].is_contiguous(), "season must be [m, N]")
    for k in ("level", "trend"):
        _vec(state[k], N, torch.float32, k, dev)
    _vec(best, N, torch.int32, "best", dev)
    _vec(sigma, N, torch.float32, "sigma", dev)
    _vec(nvalid, N, torch.float32, "nvalid", dev)
    _need(grid.dim() == 2 and grid.shape[1] == 3 and grid.dtype == torch.float32 and grid.is_contiguous()
          and grid.device == dev, "grid must be contiguous float32 [G, 3] on device")
    out = {} if out is None else out
    a = HwUpdateArgs()
    a.hist, a.ld, a.ring_len, a.col0, a.npts = nat.ptr(hist), hist.stride(0), R, int(col0), int(npts)
    a.t_last, a.m, a.N, a.bf16 = int(t_last), int(m), N, int(hist.dtype == torch.bfloat16)
    a.grid, a.best = nat.ptr(grid), nat.ptr(best)
    a.level, a.trend, a.season = nat.ptr(state["level"]), nat.ptr(state["trend"]), nat.ptr(state["season"])
    a.sigma, a.nvalid = nat.ptr(sigma), nat.ptr(nvalid)
    _fill_detect(a.det, det, N, dev, out)
    _set_hvar(a.det, det, grid, MODE_HW, m)
    nat.check(lib.fm_hw_update_detect(C.byref(a), nat.stream_handle(dev)), "fm_hw_update_detect")
    return out


# ---------------------------------------------------------------------------------
# one-shot job windows (brain/rollout.py)
# ---------------------------------------------------------------------------------

nat.register("fm_rollout_scatter", [C.c_void_p, C.c_longlong, C.c_int, C.c_int, C.c_void_p, C.c_longlong, C.c_int,
                                    C.c_longlong, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p])


def rollout_scatter(win: torch.Tensor, P: int, Wc: int, src: torch.Tensor, col0: torch.Tensor,
                    srcmap: Optional[torch.Tensor] = None) -> None:
    """``win[n, p*Wc + col0[n] + j] = src[srcmap[n*P + p], j]`` (``srcmap`` None:
    row ``n*P + p``) for the columns inside ``[0, Wc)``, mapped pods and non-NaN
    values (csrc/ingest.hip ``rollout_scatter_kernel``)."""
    lib = nat.require()
    _cuda(win, "win")
    N = win.shape[0]
    _need(win.dim() == 2 and win.dtype == torch.float32 and win.stride(1) == 1 and win.shape[1] == P * Wc,
          f"win must be float32 [N, {P * Wc}] with unit inner stride")
    _need(src.dim() == 2 and src.dtype == torch.float32 and src.stride(1) == 1 and src.device == win.device,
          "src must be float32 [S, k] on the device")
    if srcmap is None:
        _need(src.shape[0] >= N * P, f"src must have >= {N * P} rows without a srcmap")
    else:
        _vec(srcmap, N * P, torch.int32, "srcmap", win.device)
    _vec(col0, N, torch.int32, "col0", win.device)
    nat.check(lib.fm_rollout_scatter(nat.ptr(win), win.stride(0), int(P), int(Wc), nat.ptr(src), src.stride(0),
                                     int(src.shape[1]), int(src.shape[0]), nat.ptr(srcmap), nat.ptr(col0), N,
                                     nat.stream_handle(win.device)), "fm_rollout_scatter")


nat.register("fm_rollout_tick_scatter", [C.c_void_p, C.c_longlong, C.c_int, C.c_int, C.c_void_p, C.c_longlong,
                                         C.c_int, C.c_longlong, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int,
                                         C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_void_p])


def rollout_tick_scatter(win: torch.Tensor, P: int, Wc: int, src: torch.Tensor, start_min: torch.Tensor,
                         tick: torch.Tensor, srcmap: Optional[torch.Tensor] = None,
                         zero: Tuple[torch.Tensor, ...] = ()) -> None:
    """The product tick's scatter (csrc/ingest.hip ``rollout_tick_scatter_kernel``):
    ``win[n, p*Wc + tick[0] - start_min[n] + j] = src[srcmap[n*P + p], j]`` inside the
    window, and every int32 tensor of ``zero`` (at most two: the per-app counters, the
    K9 list count) zeroed in the same launch.  ``tick``: int32 device tensor whose
    element 0 is the block's first minute (read on the device: graph-capturable)."""
    lib = nat.require()
    _cuda(win, "win")
    N = win.shape[0]
    dev = win.device
    _need(win.dim() == 2 and win.dtype == torch.float32 and win.stride(1) == 1 and win.shape[1] == P * Wc,
          f"win must be float32 [N, {P * Wc}] with unit inner stride")
    _need(src.dim() == 2 and src.dtype == torch.float32 and src.stride(1) == 1 and src.device == dev,
          "src must be float32 [S, k] on the device")
    if srcmap is None:
        _need(src.shape[0] >= N * P, f"src must have >= {N * P} rows without a srcmap")
    else:
        _vec(srcmap, N * P, torch.int32, "srcmap", dev)
    _vec(start_min, N, torch.int32, "start_min", dev)
    _need(tick.dtype == torch.int32 and tick.numel() >= 1 and tick.device == dev, "tick must be int32 on the device")
    _need(len(zero) <= 2, "at most two tensors to zero")
    zs = []
    for z in zero:
        _need(z.dtype == torch.int32 and z.is_contiguous() and z.device == dev, "zeroed tensors: contiguous int32")
        zs.append((nat.ptr(z), int(z.numel())))
    while len(zs) < 2:
        zs.append((None, 0))
    nat.check(lib.fm_rollout_tick_scatter(nat.ptr(win), win.stride(0), int(P), int(Wc), nat.ptr(src), src.stride(0),
                                          int(src.shape[1]), int(src.shape[0]), nat.ptr(srcmap), nat.ptr(start_min),
                                          nat.ptr(tick), N, zs[0][0], zs[0][1], zs[1][0], zs[1][1],
                                          nat.stream_handle(dev)), "fm_rollout_tick_scatter")

