"""Host side of the fused LSTM-AE kernel (``csrc/lstm.hip``): weight packing
into MFMA A-fragment order, fp8 quantisation, launcher."""

from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Dict, List, Optional

import torch

from . import _native as nat
from .kernels import KernelShapeError, _need

H = 64
TILES, KSTEPS, KAUG = 8, 5, 80
BIAS_K = 71  # bias column of the augmented weight (k-step 4, lane half 0, element 7)
# fp8 scoring (CDNA4 v_mfma_scale_f32_32x32x64_f8f6f4): 2 k-steps of K = 64 per gate tile,
# fragments [TILES][2][64][32] e4m3 + one E8M0 scale per (tile, k-step, gate row, 32-k block),
# stored lane-major [64 lanes][16] (block b of row r in lane r + 32 b)
KSTEPS_FP8 = 2
FP8_FRAG_BYTES = TILES * KSTEPS_FP8 * 64 * 32
FP8_SCALE_BYTES = TILES * KSTEPS_FP8 * 64


class LstmRingSrc(C.Structure):
    _fields_ = [("ring", C.c_void_p * 7), ("ld", C.c_longlong), ("ring_len", C.c_int), ("bf16", C.c_int),
                ("start_col", C.c_int), ("_pad", C.c_int), ("win_series", C.c_void_p), ("win_start", C.c_void_p),
                ("mean", C.c_void_p), ("rstd", C.c_void_p), ("head_dev", C.c_void_p)]


@dataclass
class RingSource:
    """Model input read by the kernels straight from the HBM history rings:
    window w, sample t = ring column ``(start + t) mod R`` of row
    ``win_series[w]`` (or w), z-scored with ``mean`` / ``rstd`` ``[N, F]``."""
    rings: list                                  # F tensors [N, R] (bf16 or fp32, unit column stride)
    start_col: int = 0
    mean: Optional[torch.Tensor] = None          # float32 [N, F]
    rstd: Optional[torch.Tensor] = None          # float32 [N, F]
    win_series: Optional[torch.Tensor] = None    # int32 [B]
    win_start: Optional[torch.Tensor] = None     # int32 [B]
    head_dev: Optional[torch.Tensor] = None      # int32 device scalar: start_col / win_start are offsets from it

    def fill(self, src: "LstmRingSrc", n_windows: int, F: int) -> None:
        r0 = self.rings[0]
        _need(len(self.rings) == F and 1 <= F <= 7, "one ring per feature (1..7)")
        _need(all(r.shape == r0.shape and r.stride() == r0.stride() and r.dtype == r0.dtype for r in self.rings),
              "rings must share shape, strides and dtype")
        _need(r0.dim() == 2 and r0.stride(1) == 1 and r0.dtype in (torch.bfloat16, torch.float32), "ring layout")
        N, R = r0.shape
        _need(self.mean is not None and self.mean.shape == (N, F) and self.mean.dtype == torch.float32
              and self.mean.is_contiguous(), "mean must be float32 [N, F]")
        _need(self.rstd is not None and self.rstd.shape == (N, F) and self.rstd.dtype == torch.float32
              and self.rstd.is_contiguous(), "rstd must be float32 [N, F]")
        if self.win_series is not None:
            _need(self.win_series.shape == (n_windows,) and self.win_series.dtype == torch.int32, "win_series")
            _need(self.win_start is not None and self.win_start.shape == (n_windows,)
                  and self.win_start.dtype == torch.int32, "win_start")
        else:
            _need(n_windows == N, "without win_series every ring row is one window")
        for f, r in enumerate(self.rings):
            src.ring[f] = r.data_ptr()
        src.ld, src.ring_len, src.bf16 = r0.stride(0), R, int(r0.dtype == torch.bfloat16)
        src.start_col = int(self.start_col) % R
        src.win_series = nat.ptr(self.win_series)
        src.win_start = nat.ptr(self.win_start)
        src.mean, src.rstd = self.mean.data_ptr(), self.rstd.data_ptr()
        if self.head_dev is not None:
            _need(self.head_dev.dtype == torch.int32 and self.head_dev.numel() >= 1
                  and self.head_dev.device == r0.device, "head_dev must be an int32 device scalar")
        src.head_dev = nat.ptr(self.head_dev)


class LstmArgs(C.Structure):
    _fields_ = [
        ("x", C.c_void_p), ("N", C.c_int), ("T", C.c_int), ("F", C.c_int), ("fp8", C.c_int),
        ("w_enc", C.c_void_p), ("w_dec", C.c_void_p), ("w_out", C.c_void_p), ("b_out", C.c_void_p),
        ("mu", C.c_float), ("sigma", C.c_float), ("threshold", C.c_void_p), ("thr_default", C.c_float),
        ("err", C.c_void_p), ("zscore", C.c_void_p), ("verdict", C.c_void_p), ("recon", C.c_void_p),
        ("app_id", C.c_void_p), ("app_stats", C.c_void_p), ("src", LstmRingSrc),
        ("cal", C.c_void_p), ("cal_ewma", C.c_float), ("zlvl", C.c_void_p), ("thr_level", C.c_float),
        ("_pad2", C.c_int),
        ("lvl_sig", C.c_void_p), ("lvl_m", C.c_int), ("lvl_E", C.c_int), ("lvl_newest", C.c_int),
        ("lvl_avail", C.c_int), ("lvl_out", C.c_void_p),
    ]


class LevelArgs(C.Structure):
    _fields_ = [("src", LstmRingSrc), ("N", C.c_int), ("F", C.c_int), ("newest", C.c_int), ("avail", C.c_int),
                ("m", C.c_int), ("L", C.c_int), ("E", C.c_int), ("K", C.c_int), ("back_step", C.c_int),
                ("sig", C.c_void_p),
                ("out", C.c_void_p), ("head_dev", C.c_void_p)]


nat.register("fm_lstm_level", [C.POINTER(LevelArgs), C.c_void_p])
nat.register("fm_lstm_level_args_size", [], C.c_longlong)
nat.register("fm_lstm_ae", [C.POINTER(LstmArgs), C.c_void_p])
nat.register("fm_lstm_lds_bytes", [C.c_int, C.c_int], C.c_size_t)
nat.register("fm_lstm_args_size", [], C.c_longlong)
nat.register("fm_fp8_convert", [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p])
nat.register("fm_mfma_scale_probe", [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int,
                                     C.c_void_p])


def gate_row_perm() -> torch.Tensor:
    """Row permutation: packed row (tile t, r) → PyTorch gate row ``gate*H + unit``."""
    rows = []
    for t in range(TILES):
        for r in range(32):
            gate, hh, q = r >> 3, (r >> 2) & 1, r & 3
            u = 16 * (t >> 1) + 8 * hh + 4 * (t & 1) + q
            rows.append(gate * H + u)
    return torch.tensor(rows, dtype=torch.long)


def _augment(w_hh: torch.Tensor, b: torch.Tensor, w_ih: Optional[torch.Tensor], F: int) -> torch.Tensor:
    A = torch.zeros(4 * H, KAUG, dtype=torch.float32)
    A[:, :H] = w_hh.detach().float().cpu()
    if w_ih is not None:
        A[:, H:H + F] = w_ih.detach().float().cpu()
    A[:, BIAS_K] = b.detach().float().cpu()
    return A


def pack_fragments(A: torch.Tensor) -> torch.Tensor:
    """``[256, 80]`` augmented weight → ``[TILES, KSTEPS, 64, 8]`` A fragments
    (lane l: row (l & 31) of the permuted tile, k = 16 s + 8 (l >> 5) + j)."""
    P = A[gate_row_perm()]  # [256, 80] permuted rows
    out = torch.empty(TILES, KSTEPS, 64, 8, dtype=A.dtype)
    lanes = torch.arange(64)
    for t in range(TILES):
        rows = P[32 * t + (lanes & 31)]  # [64, 80]
        for s in range(KSTEPS):
            k0 = 16 * s + 8 * (lanes >> 5)  # [64]
            idx = k0[:, None] + torch.arange(8)[None, :]
            out[t, s] = rows.gather(1, idx)
    return out


_IDX_CACHE: Dict[str, torch.Tensor] = {}


def h_units(hh: torch.Tensor) -> torch.Tensor:
    """``[len(hh), 32]`` hidden unit held in h-register j of a lane of half ``hh``
    (unit 16 (tt >> 1) + 8 hh + 4 (tt & 1) + q for j = 4 tt + q): the fp8 B
    fragment's k order, so h never moves between lanes."""
    j = torch.arange(32)
    tt, q = j // 4, j % 4
    return 16 * (tt >> 1)[None, :] + 8 * hh[:, None] + 4 * (tt & 1)[None, :] + q[None, :]


def _fp8_index(device) -> torch.Tensor:
    """Flat gather index into a row-major [256, 80] augmented weight giving the
    block-scaled fp8 fragments ``[TILES, 2, 64, 32]`` (-1: zero): lane l holds
    permuted gate row 32 t + (l & 31); k-step 0, byte j: the unit of h-register j
    of lane half l >> 5; k-step 1, lane half 0: inputs at bytes 0..6 (zero weights
    past F), the bias at byte 7."""
    key = f"fp8:{device}"
    idx = _IDX_CACHE.get(key)
    if idx is None:
        rows = gate_row_perm()
        lanes = torch.arange(64)
        hh = lanes >> 5
        unit = h_units(hh)                                  # [64, 32]
        j = torch.arange(32)[None, :]
        out = torch.empty(TILES, KSTEPS_FP8, 64, 32, dtype=torch.long)
        for t in range(TILES):
            r = rows[32 * t + (lanes & 31)][:, None]         # [64, 1]
            out[t, 0] = r * KAUG + unit
            out[t, 1] = torch.where((hh[:, None] == 0) & (j < 8), r * KAUG + H + j, torch.full_like(j, -1))
        idx = out.flatten().to(device)
        _IDX_CACHE[key] = idx
    return idx


def pack_fp8(A: torch.Tensor) -> torch.Tensor:
    """``[256, 80]`` augmented weight → the fp8 kernel's uint8 buffer: block-scaled
    e4m3 fragments ``[TILES, 2, 64, 32]`` stored half-major (one scale per gate row and
    32-k block),
    then the E8M0 scales ``[64 lanes, 16]``
    (:func:`~foremast_amd.ops.pack.fp8_blocks_lane_major`)."""
    from .pack import fp8_blocks_lane_major
    idx = _fp8_index(A.device)
    v = torch.where(idx >= 0, A.float().flatten()[idx.clamp(min=0)], torch.zeros((), device=A.device))
    return fp8_blocks_lane_major(v)


def _frag_index(device) -> torch.Tensor:
    """Flat gather index into a row-major [256, 80] augmented weight that
    produces the A-fragment layout (device-side repacking every train step)."""
    key = str(device)
    idx = _IDX_CACHE.get(key)
    if idx is None:
        rows = gate_row_perm()
        lanes = torch.arange(64)
        out = torch.empty(TILES, KSTEPS, 64, 8, dtype=torch.long)
        for t in range(TILES):
            r = rows[32 * t + (lanes & 31)]
            for s in range(KSTEPS):
                k = 16 * s + 8 * (lanes >> 5)
                out[t, s] = r[:, None] * KAUG + k[:, None] + torch.arange(8)[None, :]
        idx = out.flatten().to(device)
        _IDX_CACHE[key] = idx
    return idx


def _augment_dev(w_hh, b, w_ih, F) -> torch.Tensor:
    A = torch.zeros(4 * H, KAUG, dtype=torch.float32, device=w_hh.device)
    A[:, :H] = w_hh.detach()
    if w_ih is not None:
        A[:, H:H + F] = w_ih.detach()
    A[:, BIAS_K] = b.detach()
    return A


# parameter order of the pack sources (csrc/pack.hip codes refer to these ids)
LSTM_SRCS = ("enc_w_hh", "enc_w_ih", "enc_b", "dec_w_hh", "dec_b", "out_w", "out_b")


def model_srcs(model) -> List[torch.Tensor]:
    return [getattr(model, n).data for n in LSTM_SRCS]


def augmented_codes(F: int, enc: bool, fp8: bool = False) -> torch.Tensor:
    """Pack codes of the A-fragment layout of ``[W_hh | W_ih | b]`` (the
    ``_augment`` + ``pack_fragments`` reference, as a table; ``fp8``: the
    block-scaled layout of :func:`_fp8_index`)."""
    from .pack import make_codes
    idx = _fp8_index("cpu") if fp8 else _frag_index("cpu")
    used = idx >= 0
    idx = idx.clamp(min=0)
    r, k = idx // KAUG, idx % KAUG
    is_h, is_b = (k < H) & used, (k == BIAS_K) & used
    is_x = (k >= H) & (k < H + F) & torch.tensor(enc) & used
    src = torch.where(is_h, LSTM_SRCS.index("enc_w_hh" if enc else "dec_w_hh"),
                      torch.where(is_b, LSTM_SRCS.index("enc_b" if enc else "dec_b"), LSTM_SRCS.index("enc_w_ih")))
    off = torch.where(is_h, r * H + k, torch.where(is_b, r, r * F + (k - H)))
    return make_codes(src, off.clamp(min=0), valid=is_h | is_b | is_x)


def identity_codes(name: str, n: int) -> torch.Tensor:
    from .pack import make_codes
    return make_codes(torch.full((n,), LSTM_SRCS.index(name)), torch.arange(n))


def scoring_packer(p: "LstmPacked", model):
    """Native packer refreshing ``p`` from ``model`` (one launch; two for fp8)."""
    from .pack import KIND_BF16, KIND_F32, KIND_FP8, Packer
    F = model.F
    kind = KIND_FP8 if p.fp8 else KIND_BF16
    pk = Packer(model_srcs(model))
    pk.add(augmented_codes(F, True, p.fp8), p.w_enc.view(-1), kind)
    pk.add(augmented_codes(F, False, p.fp8), p.w_dec.view(-1), kind)
    pk.add(identity_codes("out_w", F * H), p.w_out.view(-1), KIND_F32)
    pk.add(identity_codes("out_b", F), p.b_out.view(-1), KIND_F32)
    return pk


def repack_into(p: "LstmPacked", model) -> "LstmPacked":
    """Refresh ``p`` in place from (device) model parameters.  With the native
    library: one table-driven pack launch (fp8: block scales computed on the
    device); otherwise torch gathers (:func:`pack_fp8` for fp8)."""
    if p.w_enc.is_cuda and nat.available():
        if p.packer is None or p.packer_model is not model:
            p.packer, p.packer_model = scoring_packer(p, model), model
        p.packer.run()
        return p
    F = model.F
    if p.fp8:
        p.w_enc.copy_(pack_fp8(_augment_dev(model.enc_w_hh, model.enc_b, model.enc_w_ih, F)))
        p.w_dec.copy_(pack_fp8(_augment_dev(model.dec_w_hh, model.dec_b, None, F)))
    else:
        idx = _frag_index(p.w_enc.device)
        Ae = _augment_dev(model.enc_w_hh, model.enc_b, model.enc_w_ih, F).flatten()[idx]
        Ad = _augment_dev(model.dec_w_hh, model.dec_b, None, F).flatten()[idx]
        p.w_enc.copy_(Ae.to(torch.bfloat16).view_as(p.w_enc))
        p.w_dec.copy_(Ad.to(torch.bfloat16).view_as(p.w_dec))
    p.w_out.copy_(model.out_w.detach())
    p.b_out.copy_(model.out_b.detach())
    return p


@dataclass
class LstmPacked:
    F: int
    fp8: bool
    w_enc: torch.Tensor   # bf16 fragments, or the fp8 buffer (block-scaled fragments + E8M0 scales)
    w_dec: torch.Tensor
    w_out: torch.Tensor
    b_out: torch.Tensor
    packer: Optional[object] = None
    packer_model: Optional[object] = None


def pack(model, fp8: bool = False, device="cuda") -> LstmPacked:
    F = model.F
    if model.H != H:
        raise KernelShapeError(f"fused LSTM kernel is built for H={H}")
    if not 1 <= F <= 7:
        raise KernelShapeError("fused LSTM kernel supports 1..7 features")
    if fp8:
        qe = pack_fp8(_augment(model.enc_w_hh, model.enc_b, model.enc_w_ih, F))
        qd = pack_fp8(_augment(model.dec_w_hh, model.dec_b, None, F))
        return LstmPacked(F=F, fp8=True, w_enc=qe.contiguous().to(device), w_dec=qd.contiguous().to(device),
                          w_out=model.out_w.detach().float().contiguous().to(device),
                          b_out=model.out_b.detach().float().contiguous().to(device))
    Ae = pack_fragments(_augment(model.enc_w_hh, model.enc_b, model.enc_w_ih, F))
    Ad = pack_fragments(_augment(model.dec_w_hh, model.dec_b, None, F))
    return LstmPacked(F=F, fp8=False, w_enc=Ae.to(torch.bfloat16).contiguous().to(device),
                      w_dec=Ad.to(torch.bfloat16).contiguous().to(device),
                      w_out=model.out_w.detach().float().contiguous().to(device),
                      b_out=model.out_b.detach().float().contiguous().to(device))


def fp8_emulated_forward(model, x: torch.Tensor):
    """The fp8 scoring kernel's arithmetic in PyTorch (fp32 everywhere else): what the
    block-scaled ``v_mfma_scale_f32_32x32x64_f8f6f4`` path quantises, it quantises the
    same way, so a comparison against it measures only accumulation order and the
    hardware transcendentals.

    * weights: e4m3 codes of ``w * 2^-e`` with one E8M0 exponent per (gate row, 32-k
      block), :func:`~foremast_amd.ops.pack.e8m0_blocks`: ``W_hh`` blocks are hidden
      units 0..31 and 32..63; the input k-step's block 0 is ``(W_ih[row, :F], 0.., b[row]
      at byte 7)`` (decoder: the bias alone);
    * the hidden state enters as ``e4m3(h * 2^8) * 2^-8``, the inputs as
      ``e4m3(clamp(x, +-448))``, the bias input as 1;
    * gates, cell, read-out (unquantised h, fp32 ``W_out``) and the error against the
      unquantised x in fp32.
    Returns ``(y [N, T, F], err [N])``."""
    from .pack import e8m0_blocks
    F = model.F
    e4 = torch.float8_e4m3fn

    def deq(blocks: torch.Tensor) -> torch.Tensor:
        q, sc = e8m0_blocks(blocks)
        return q.view(e4).float() * torch.ldexp(torch.ones_like(sc, dtype=torch.float32),
                                                 (sc.int() - 127))[:, None]

    def hh_hat(w):  # [4H, H] -> per (row, 32-unit block)
        return deq(w.detach().float().cpu().reshape(4 * H * 2, 32)).reshape(4 * H, H)

    def in_block(w_ih, b):  # [4H, 32]: inputs at 0..F-1, bias at 7
        blk = torch.zeros(4 * H, 32)
        if w_ih is not None:
            blk[:, :F] = w_ih.detach().float().cpu()
        blk[:, 7] = b.detach().float().cpu()
        d = deq(blk)
        return (d[:, :F] if w_ih is not None else None), d[:, 7]

    we_hh, wd_hh = hh_hat(model.enc_w_hh), hh_hat(model.dec_w_hh)
    we_ih, be = in_block(model.enc_w_ih, model.enc_b)
    _, bd = in_block(None, model.dec_b)
    x = x.detach().float().cpu()
    N, T, _ = x.shape
    xq = x.clamp(-448.0, 448.0).to(e4).float()

    def hq(h):
        return (h * 256.0).to(e4).float() / 256.0

    cell = type(model)._cell
    h = torch.zeros(N, H)
    c = torch.zeros(N, H)
    for t in range(T):
        h, c = cell(hq(h) @ we_hh.t() + xq[:, t] @ we_ih.t() + be, c)
    ys = []
    for t in range(T):
        h, c = cell(hq(h) @ wd_hh.t() + bd, c)
        ys.append(h)
    y = torch.stack(ys, 1) @ model.out_w.detach().float().cpu().t() + model.out_b.detach().float().cpu()
    return y, ((y - x) ** 2).mean(dim=(1, 2))


def lstm_score(p: LstmPacked, x: Optional[torch.Tensor], mu: float = 0.0, sigma: float = 1.0,
               threshold: Optional[torch.Tensor] = None, thr_default: float = 3.0, want_recon: bool = False,
               app_id: Optional[torch.Tensor] = None, app_stats: Optional[torch.Tensor] = None,
               out: Optional[Dict[str, torch.Tensor]] = None, ring: Optional[RingSource] = None,
               T: Optional[int] = None, cal: Optional[torch.Tensor] = None,
               cal_ewma: float = 0.0, zlvl: Optional[torch.Tensor] = None,
               thr_level: float = float("inf"), level: Optional[Dict] = None) -> Dict[str, torch.Tensor]:
    """Score windows ``x [N, T, F]`` — or, with ``ring`` (and ``T``), the last
    ``T`` samples of every ring row (or the ``ring.win_series`` / ``win_start``
    windows) read directly by the kernel.

    ``cal`` ``[N, 2]`` float32 (per-window ``mu``, ``1/sigma``): the z-score is
    the smaller of the global one (``mu``/``sigma``) and the window's own
    series' one, so a window must be unusual for its series AND in absolute
    terms; with ``cal_ewma > 0`` the kernel moves ``mu`` toward every
    non-anomalous error (relative dispersion kept).  ``zlvl`` ``[N, F]`` (from
    :func:`lstm_level`): a window is also anomalous when any ``|zlvl|`` exceeds
    ``thr_level``.  ``level`` (ring input, one window per row): the kernel computes the
    level z itself (:func:`lstm_level`'s statistic) — ``{"sig": [N, F] spread, "m":
    samples per day, "newest": newest column (an offset from ``ring.head_dev`` when set),
    "avail": valid samples, "E": extra points (default :func:`level_extension`),
    "out": optional [N, F] z}``."""
    lib = nat.require()
    if ring is None:
        _need(x is not None and x.is_cuda and x.dtype == torch.float32 and x.dim() == 3 and x.is_contiguous(),
              "x must be a contiguous float32 [N, T, F] GPU tensor")
        N, T, F = x.shape
        dev = x.device
    else:
        _need(T is not None and T >= 1, "ring scoring needs the window length T")
        F = len(ring.rings)
        N = ring.win_series.shape[0] if ring.win_series is not None else ring.rings[0].shape[0]
        dev = ring.rings[0].device
    _need(F == p.F, f"feature mismatch {F} vs {p.F}")
    if threshold is not None:
        _need(threshold.shape == (N,) and threshold.dtype == torch.float32 and threshold.is_contiguous()
              and threshold.device == dev, "threshold must be float32 [N]")
    if app_id is not None:
        _need(app_id.shape == (N,) and app_id.dtype == torch.int32 and app_stats is not None
              and app_stats.dtype == torch.int32 and app_stats.is_contiguous(), "app_id/app_stats")
    if cal is not None:
        _need(cal.shape == (N, 2) and cal.dtype == torch.float32 and cal.is_contiguous() and cal.device == dev,
              "cal must be float32 [N, 2] (mu, 1/sigma)")
    out = {} if out is None else out
    out.setdefault("err", torch.empty(N, dtype=torch.float32, device=dev))
    out.setdefault("zscore", torch.empty(N, dtype=torch.float32, device=dev))
    out.setdefault("verdict", torch.empty(N, dtype=torch.int8, device=dev))
    if want_recon:
        out.setdefault("recon", torch.empty((N, T, F), dtype=torch.float32, device=dev))
    a = LstmArgs()
    a.x = 0 if x is None else x.data_ptr()
    if ring is not None:
        ring.fill(a.src, N, F)
    a.N, a.T, a.F, a.fp8 = N, T, F, int(p.fp8)
    a.w_enc, a.w_dec = p.w_enc.data_ptr(), p.w_dec.data_ptr()
    a.w_out, a.b_out = p.w_out.data_ptr(), p.b_out.data_ptr()
    a.mu, a.sigma = float(mu), float(sigma)
    a.threshold = nat.ptr(threshold)
    a.thr_default = float(thr_default)
    a.err, a.zscore, a.verdict = nat.ptr(out["err"]), nat.ptr(out["zscore"]), nat.ptr(out["verdict"])
    a.recon = nat.ptr(out.get("recon")) if want_recon else 0
    a.app_id, a.app_stats = nat.ptr(app_id), nat.ptr(app_stats)
    a.cal, a.cal_ewma = nat.ptr(cal), float(cal_ewma)
    if level is not None:
        _need(ring is not None and ring.win_series is None, "the fused level term reads the rings, one window per row")
        sig, R = level["sig"], ring.rings[0].shape[1]
        _need(sig.shape == (N, F) and sig.dtype == torch.float32 and sig.is_contiguous() and sig.device == dev,
              "level sig must be float32 [N, F]")
        m, newest, avail = int(level["m"]), int(level["newest"]), int(level["avail"])
        E = level_extension(m) if level.get("E") is None else int(level["E"])
        _need(0 <= newest < R and 0 < avail <= R and 0 <= E <= 12 and m >= 8 + 2 * E, "level geometry")
        lo = level.get("out")
        if lo is not None:
            _need(lo.shape == (N, F) and lo.dtype == torch.float32 and lo.is_contiguous(), "level out [N, F]")
        a.lvl_sig, a.lvl_m, a.lvl_E, a.lvl_newest, a.lvl_avail = sig.data_ptr(), m, E, newest, avail
        a.lvl_out = nat.ptr(lo)
    if zlvl is not None:
        _need(zlvl.shape == (N, F) and zlvl.dtype == torch.float32 and zlvl.is_contiguous() and zlvl.device == dev,
              "zlvl must be float32 [N, F]")
    a.zlvl, a.thr_level = nat.ptr(zlvl), float(thr_level)
    nat.check(lib.fm_lstm_ae(C.byref(a), nat.stream_handle(dev)), "fm_lstm_ae")
    return out


def level_extension(m: int) -> int:
    """Extra minutes each side of the earlier days' windows for a season of ``m``
    samples: 12 for a day of minutes, fewer when the profile's curvature over the
    window would bias the centred mean."""
    return max(0, min(12, int(round(m / 120))))


def lstm_level(rings: List[torch.Tensor], newest: int, avail: int, m: int, L: int = 8,
               sig: Optional[torch.Tensor] = None, K: int = 0, back_step: int = 0,
               out: Optional[torch.Tensor] = None, E: Optional[int] = None,
               head_dev: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Level statistic of every (row, feature) (see ``LevelArgs`` in csrc/lstm.hip):
    the mean over the newest ``L`` samples of x_t minus the same minutes' mean over
    up to 7 earlier days.  Scoring (``K == 0``): ``[N, F]`` statistic / ``sig``.
    Calibration: the raw statistic ``[K, N, F]`` at offsets ending ``(k+1) *
    back_step`` samples before the newest (NaN where a window has no data)."""
    lib = nat.require()
    F = len(rings)
    r0 = rings[0]
    _need(1 <= F <= 7 and all(r.shape == r0.shape and r.stride() == r0.stride() and r.dtype == r0.dtype
                              for r in rings), "one ring per feature, same layout")
    _need(r0.dim() == 2 and r0.stride(1) == 1 and r0.dtype in (torch.bfloat16, torch.float32), "ring layout")
    N, R = r0.shape
    E = level_extension(m) if E is None else int(E)
    _need(0 <= newest < R and L == 8 and 0 <= E <= 12 and m >= L + 2 * E, "level geometry")
    dev = r0.device
    if K == 0:
        _need(sig is not None and sig.shape == (N, F) and sig.dtype == torch.float32 and sig.is_contiguous(),
              "sig must be float32 [N, F]")
        shape = (N, F)
    else:
        _need(back_step >= 1 and K <= 65535, "calibration offsets")
        shape = (K, N, F)
    if out is None or out.shape != shape:
        out = torch.empty(shape, dtype=torch.float32, device=dev)
    a = LevelArgs()
    for f, r in enumerate(rings):
        a.src.ring[f] = r.data_ptr()
    a.src.ld, a.src.ring_len, a.src.bf16 = r0.stride(0), R, int(r0.dtype == torch.bfloat16)
    a.N, a.F, a.newest, a.avail, a.m, a.L, a.E, a.K, a.back_step = N, F, int(newest), int(avail), int(m), int(L), \
        E, int(K), int(back_step)
    a.sig, a.out = nat.ptr(sig), out.data_ptr()
    if head_dev is not None:  # graph-captured ticks: `newest` is an offset from the device head
        _need(head_dev.dtype == torch.int32 and head_dev.numel() >= 1 and head_dev.device == dev,
              "head_dev must be an int32 device scalar")
    a.head_dev = nat.ptr(head_dev)
    nat.check(lib.fm_lstm_level(C.byref(a), nat.stream_handle(dev)), "fm_lstm_level")
    return out


def device_fp8(values: torch.Tensor) -> torch.Tensor:
    """Convert with the device's ``v_cvt_pk_fp8_f32`` (format agreement tests)."""
    lib = nat.require()
    v = values.float().contiguous()
    out = torch.empty(v.numel(), dtype=torch.uint8, device=v.device)
    nat.check(lib.fm_fp8_convert(v.data_ptr(), out.data_ptr(), v.numel(), nat.stream_handle(v.device)),
              "fm_fp8_convert")
    return out


def mfma_scale_probe(A: torch.Tensor, B: torch.Tensor, sa_reg: torch.Tensor, sb_reg: torch.Tensor,
                     sel: int = 0) -> torch.Tensor:
    """ONE ``v_mfma_scale_f32_32x32x64_f8f6f4`` on e4m3 data: lane l holds row / column
    ``l & 31`` of ``A [32, 64]`` / ``B [64, 32]`` (float32, converted on the device) at
    k = 32 (l >> 5) + j, and passes ``sa_reg[l]`` / ``sb_reg[l]`` (int32 [64]) as its
    scale registers with op_sel ``sel``; returns D [32, 32]."""
    lib = nat.require()
    _need(A.shape == (32, 64) and B.shape == (64, 32) and sa_reg.shape == (64,) and sb_reg.shape == (64,),
          "probe shapes: A [32, 64], B [64, 32], scale registers [64]")
    A, B = A.float().contiguous(), B.float().contiguous()
    sa, sb = sa_reg.to(torch.int32).contiguous(), sb_reg.to(torch.int32).contiguous()
    _need(A.is_cuda and all(t.device == A.device for t in (B, sa, sb)), "probe tensors on one GPU")
    D = torch.empty((32, 32), dtype=torch.float32, device=A.device)
    nat.check(lib.fm_mfma_scale_probe(A.data_ptr(), B.data_ptr(), sa.data_ptr(), sb.data_ptr(), D.data_ptr(),
                                      int(sel), nat.stream_handle(A.device)), "fm_mfma_scale_probe")
    return D
