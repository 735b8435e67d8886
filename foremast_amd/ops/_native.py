"""ctypes binding to ``_lib/libforemast_hip.so`` (the gfx950 kernels).

The library's only dependency is ``libamdhip64.so.7``; PyTorch-ROCm ships a
runtime with the same soname, so we import torch first and the dynamic
loader reuses torch's HIP runtime — our kernels run on torch's streams and
read torch's allocations directly.

On a GPU box a missing or stale library is a hard error (no silent
fall-back): ``require()`` raises with the build command to run.
"""

from __future__ import annotations

import ctypes as C
import os
import threading
from typing import Optional

import torch  # noqa: F401  (must be loaded before the HIP library)

from . import build as _build

_lock = threading.Lock()
_lib: Optional[C.CDLL] = None
_err: Optional[str] = None

P = C.c_void_p
I = C.c_int
LL = C.c_longlong
F = C.c_float


class DetectArgs(C.Structure):
    _fields_ = [
        ("horizons", P), ("h_ld", LL), ("C", I), ("min_valid", I),
        ("cur", P), ("ld_cur", LL),
        ("threshold", P), ("bound", P), ("min_lower", P), ("differs", P),
        ("pw_scale", F), ("pw_min_points", I), ("threshold_low", P),
        ("hv_grid", P), ("hv_mode", I), ("hv_m", I),
        ("forecast", P), ("upper", P), ("lower", P), ("count", P), ("verdict", P),
        ("score", P), ("app_id", P), ("app_stats", P),
        ("anom_count", P), ("anom_series", P), ("anom_col", P), ("anom_val", P), ("anom_cap", I), ("shift_thr", F), ("base_mean", P),
        ("shift_min_points", I), ("shift_one_step", I),
        ("thr_lut", P), ("thr_cls", P), ("lut_n", I), ("last_ncol", I), ("row_out", P), ("start_min", P),
        ("tick_min", P),
    ]


class SmoothArgs(C.Structure):
    _fields_ = [
        ("hist", P), ("ld", LL), ("ring_len", I), ("head", I), ("T", I), ("Tp", I),
        ("pad", I), ("m", I), ("K", I), ("seg", I), ("grid", P), ("G", I), ("N", I),
        ("level", P), ("trend", P), ("sigma", P), ("best", P), ("season_out", P),
        ("pair_tab", P), ("det", DetectArgs), ("head_dev", P), ("season_hb", P), ("nvalid_out", P),
    ]


class RankArgs(C.Structure):
    _fields_ = [
        ("base", P), ("ld_base", LL), ("cur", P), ("ld_cur", LL),
        ("nb", I), ("nc", I), ("N", I), ("mode", I), ("alpha", F),
        ("min_mw", I), ("min_wilcoxon", I), ("min_kruskal", I),
        ("pvals", P), ("differs", P), ("counts", P),
        ("pods_b", I), ("pods_c", I), ("min_friedman", I), ("p_friedman", P), ("base_mean", P),
        ("z_crit", F), ("_pad", I),
    ]


class WindowArgs(C.Structure):
    _fields_ = [
        ("hist", P), ("ld", LL), ("ring_len", I), ("head", I), ("len", I), ("N", I),
        ("mean", P), ("stdv", P), ("count", P), ("det", DetectArgs),
    ]


class BivArgs(C.Structure):
    _fields_ = [
        ("hx", P), ("hy", P), ("ld", LL), ("ring_len", I), ("head", I), ("len", I), ("N", I),
        ("cur", P), ("C", I), ("min_valid", I), ("threshold", P), ("differs", P),
        ("pw_scale", F), ("eps", F), ("mean", P), ("cov", P), ("d2", P), ("count", P),
        ("verdict", P), ("score", P), ("app_id", P), ("app_stats", P),
    ]


class LstmArgs(C.Structure):
    pass  # populated in lstm bindings (see kernels.py)


def _declare(lib: C.CDLL) -> None:
    lib.fm_smooth_fit.argtypes = [C.POINTER(SmoothArgs), I, I, I, P]
    lib.fm_smooth_fit.restype = I
    lib.fm_smooth_lds_bytes.argtypes = [I, I, I, I]
    lib.fm_smooth_lds_bytes.restype = C.c_size_t
    lib.fm_hw_scan_lds_bytes.argtypes = [I, I, I, I, I]
    lib.fm_hw_scan_lds_bytes.restype = C.c_size_t
    lib.fm_hw_half_lds_bytes.argtypes = [I, I, I]
    lib.fm_hw_half_lds_bytes.restype = C.c_size_t
    lib.fm_hw_half_fit.argtypes = [C.POINTER(SmoothArgs), I, P, P]
    lib.fm_hw_half_fit.restype = I
    lib.fm_hw_d_lds_bytes.argtypes = [I, I, I]
    lib.fm_hw_d_lds_bytes.restype = C.c_size_t
    lib.fm_hw_d_fit.argtypes = [C.POINTER(SmoothArgs), I, P, P]
    lib.fm_hw_d_fit.restype = I
    lib.fm_hw_d_fit_split.argtypes = [C.POINTER(SmoothArgs), I, P, P, I, I, P]
    lib.fm_hw_d_fit_split.restype = I
    lib.fm_hw_q_lds_bytes.argtypes = [I, I, I]
    lib.fm_hw_q_lds_bytes.restype = C.c_size_t
    lib.fm_hw_q_fit.argtypes = [C.POINTER(SmoothArgs), P, I, P, P]
    lib.fm_hw_q_fit.restype = I
    lib.fm_hw_d_split_plan.argtypes = [I, I, I]
    lib.fm_hw_d_split_plan.restype = I
    lib.fm_es_seq_fit.argtypes = [C.POINTER(SmoothArgs), I, I, P]
    lib.fm_es_seq_fit.restype = I
    lib.fm_es_seq_tpc.argtypes = [I]
    lib.fm_es_seq_tpc.restype = I
    lib.fm_hw_seq_fit.argtypes = [C.POINTER(SmoothArgs), I, P]
    lib.fm_hw_seq_fit.restype = I
    lib.fm_hw_seq_lds_bytes.argtypes = [I, I, I]
    lib.fm_hw_seq_lds_bytes.restype = C.c_size_t
    lib.fm_hw_seq_tpc.argtypes = [I, I]
    lib.fm_hw_seq_tpc.restype = I
    lib.fm_hw_detect_params.argtypes = [C.POINTER(SmoothArgs), P]
    lib.fm_hw_detect_params.restype = I
    lib.fm_rank_tests.argtypes = [C.POINTER(RankArgs), P]
    lib.fm_rank_tests.restype = I
    lib.fm_rank_lds_bytes.argtypes = [I, I]
    lib.fm_rank_lds_bytes.restype = C.c_size_t
    lib.fm_window_stats.argtypes = [C.POINTER(WindowArgs), I, P]
    lib.fm_window_stats.restype = I
    lib.fm_bivariate.argtypes = [C.POINTER(BivArgs), I, P]
    lib.fm_bivariate.restype = I
    lib.fm_ring_append.argtypes = [P, LL, I, I, I, P, LL, LL, I, P]
    lib.fm_ring_append.restype = I
    lib.fm_ring_append_dev.argtypes = [P, LL, I, I, P, I, P, LL, LL, I, P]
    lib.fm_ring_append_dev.restype = I
    lib.fm_tick_ingest.argtypes = [P, LL, I, P, LL, I, I, I, P, LL, I, I, P, P, I, P, I, P]
    lib.fm_tick_ingest.restype = I
    lib.fm_tick_ingest_dev.argtypes = [P, LL, P, LL, I, I, P, LL, I, P, P, I, P, P, I, P]
    lib.fm_tick_ingest_dev.restype = I
    lib.fm_copy_to_host_i32.argtypes = [P, P, LL, P]
    lib.fm_copy_to_host_i32.restype = I
    lib.fm_tick_advance.argtypes = [P, I, I, P, I, P, P, P, LL, P]
    lib.fm_tick_advance.restype = I
    for name, args in _EXTRA.items():
        fn = getattr(lib, name, None)
        if fn is not None:
            fn.argtypes = args[0]
            fn.restype = args[1]


# additional symbols registered by other modules (e.g. LSTM, compaction)
_EXTRA = {}


def register(name: str, argtypes, restype=I) -> None:
    _EXTRA[name] = (argtypes, restype)
    if _lib is not None:
        fn = getattr(_lib, name, None)
        if fn is not None:
            fn.argtypes = argtypes
            fn.restype = restype


def load(build_if_missing: bool = False) -> Optional[C.CDLL]:
    global _lib, _err
    with _lock:
        if _lib is not None:
            return _lib
        path = _build.lib_path()
        if not os.path.exists(path) and build_if_missing:
            try:
                _build.build()
            except Exception as e:  # pragma: no cover - toolchain issues
                _err = str(e)
                return None
        if not os.path.exists(path):
            _err = f"{path} not built (run: python -m foremast_amd.ops.build)"
            return None
        try:
            lib = C.CDLL(path, mode=C.RTLD_GLOBAL)
        except OSError as e:
            _err = f"failed to load {path}: {e}"
            return None
        _declare(lib)
        _lib = lib
        return lib


def available() -> bool:
    return load() is not None


def require() -> C.CDLL:
    lib = load(build_if_missing=True)
    if lib is None:
        raise RuntimeError(f"foremast HIP kernels unavailable: {_err}")
    return lib


def check(code: int, what: str) -> None:
    if code != 0:
        raise RuntimeError(f"{what} failed with hipError {code}")


def ptr(t) -> int:
    return 0 if t is None else int(t.data_ptr())


def stream_handle(device=None) -> int:
    return int(torch.cuda.current_stream(device).cuda_stream)
