"""Host side of the fused LSTM-AE training kernel (``csrc/lstm_train.hip``).

:class:`FusedLstmGrad` computes the gradient of ``model.recon_error(x).mean()``
for every parameter of an :class:`~foremast_amd.models.lstm_ae.LSTMAutoencoder`
(H = 64) in one kernel launch plus three hipBLASLt GEMMs, and writes it into
``p.grad`` (which, under :class:`~foremast_amd.parallel.dp.DPTrainer`, are views
into the flat all-reduce buckets).  Weights are repacked on the device every
call (forward A fragments as in :mod:`.lstm`, plus ``W_hh^T`` fragments for the
backward recurrence).
"""

from __future__ import annotations

import ctypes as C
import os
from typing import Dict, Optional

import torch

from . import _native as nat
from .kernels import KernelShapeError, _need
from .lstm import BIAS_K, H, KAUG, LstmRingSrc, RingSource, _augment_dev, _frag_index


class LstmTrainArgs(C.Structure):
    _fields_ = [
        ("x", C.c_void_p), ("B", C.c_int), ("T", C.c_int), ("F", C.c_int), ("phases", C.c_int),
        ("w_enc", C.c_void_p), ("w_dec", C.c_void_p), ("wt_enc", C.c_void_p), ("wt_dec", C.c_void_p),
        ("w_out", C.c_void_p), ("b_out", C.c_void_p), ("scratch", C.c_void_p),
        ("g_enc", C.c_void_p), ("g_dec", C.c_void_p), ("h_enc", C.c_void_p), ("h_dec", C.c_void_p),
        ("dy", C.c_void_p), ("err", C.c_void_p), ("loss_scale", C.c_float), ("variant", C.c_int),
        ("src", LstmRingSrc),
    ]


nat.register("fm_lstm_ae_train", [C.POINTER(LstmTrainArgs), C.c_void_p])
nat.register("fm_lstm_train_lds_bytes", [C.c_int], C.c_size_t)
nat.register("fm_lstm_train_scratch_floats", [C.c_int, C.c_int], C.c_longlong)
nat.register("fm_lstm_train_args_size", [], C.c_longlong)


def _unit(tile, hh, q):
    return 16 * (tile >> 1) + 8 * hh + 4 * (tile & 1) + q


def transposed_frag_index() -> torch.Tensor:
    """Flat gather index into a row-major ``W_hh [256, 64]`` giving the backward
    A fragments ``[2 M-tiles][16 k-steps][64 lanes][8]``: lane l, element j of
    (mt, ks) holds ``W_hh[p][u]`` with ``p`` the gate row carried by forward
    accumulator register ``r = 8 (ks & 1) + j`` of tile ``ks >> 1`` in lane half
    ``l >> 5`` and ``u`` the hidden unit whose dh lands in accumulator row
    ``l & 31`` of M-tile ``mt`` (= h register ``16 mt + r'``)."""
    idx = torch.empty(2, 16, 64, 8, dtype=torch.long)
    for mt in range(2):
        for ks in range(16):
            tt, e = ks >> 1, ks & 1
            for lane in range(64):
                hk, m = lane >> 5, lane & 31
                u = _unit(4 * mt + (m >> 3), (m >> 2) & 1, m & 3)
                for j in range(8):
                    r = 8 * e + j
                    p = (r >> 2) * H + _unit(tt, hk, r & 3)
                    idx[mt, ks, lane, j] = p * H + u
    return idx.flatten()


_T_IDX: Dict[str, torch.Tensor] = {}


def _t_index(device) -> torch.Tensor:
    k = str(device)
    if k not in _T_IDX:
        _T_IDX[k] = transposed_frag_index().to(device)
    return _T_IDX[k]


def _bmm_sum_f32(a: torch.Tensor, b: torch.Tensor, chunks: int) -> torch.Tensor:
    """``a [M, K] @ b [K, N]`` as a strided-batched GEMM over ``chunks`` K-slices
    summed in fp32: the K = T*B reduction of the weight gradients is far too
    deep for one tall-skinny GEMM to fill the GPU; T slices of K = B run as one
    batched launch (no copies: the slices are strided views)."""
    M, K = a.shape
    N = b.shape[1]
    kc = K // chunks
    av = a.as_strided((chunks, M, kc), (kc, a.stride(0), a.stride(1)))
    bv = b.as_strided((chunks, kc, N), (kc * b.stride(0), b.stride(0), b.stride(1)))
    try:
        return torch.bmm(av, bv, out_dtype=torch.float32).sum(0)
    except (RuntimeError, TypeError, NotImplementedError):
        return torch.bmm(av.float(), bv.float()).sum(0)


def _mm_f32(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """bf16 x bf16 → fp32 GEMM (hipBLASLt) without rounding the result to bf16."""
    try:
        return torch.mm(a, b, out_dtype=torch.float32)
    except (RuntimeError, TypeError, NotImplementedError):
        return torch.mm(a.float(), b.float())


class FusedLstmGrad:
    """Reusable buffers + launcher for one (B, T, F) training shape."""

    def __init__(self, B: int, T: int, F: int, device, variant: Optional[int] = None) -> None:
        """``variant`` 0: one wave per 32 windows; 1 (default): two waves per 32
        windows splitting the hidden units (env ``FOREMAST_LSTM_TRAIN_VARIANT``)."""
        self.variant = int(os.environ.get("FOREMAST_LSTM_TRAIN_VARIANT", "1")) if variant is None else int(variant)
        if B % 32:
            raise KernelShapeError("fused LSTM training needs B % 32 == 0")
        if not 1 <= F <= 7:
            raise KernelShapeError("fused LSTM training supports 1..7 features")
        lib = nat.require()
        self.B, self.T, self.F = B, T, F
        dev = torch.device(device)
        self.device = dev
        KB = T * B
        self.scratch = torch.empty(int(lib.fm_lstm_train_scratch_floats(B, T)), dtype=torch.float32, device=dev)
        # K-contiguous [rows, T*B] operands of the weight-gradient GEMMs
        self.g_enc = torch.empty((4 * H, KB), dtype=torch.bfloat16, device=dev)
        self.g_dec = torch.empty((4 * H, KB), dtype=torch.bfloat16, device=dev)
        self.h_enc = torch.zeros((KAUG, KB), dtype=torch.bfloat16, device=dev)
        self.h_dec = torch.zeros((KAUG, KB + B), dtype=torch.bfloat16, device=dev)
        self.h_enc[BIAS_K] = 1.0
        self.h_dec[BIAS_K] = 1.0
        self.dy = torch.empty((F, KB), dtype=torch.float32, device=dev)
        self.err = torch.empty(B, dtype=torch.float32, device=dev)
        self.w_enc = torch.empty(8 * 5 * 64 * 8, dtype=torch.bfloat16, device=dev)
        self.w_dec = torch.empty_like(self.w_enc)
        self.wt_enc = torch.empty(2 * 16 * 64 * 8, dtype=torch.bfloat16, device=dev)
        self.wt_dec = torch.empty_like(self.wt_enc)

    def _packer_for(self, model):
        """Native packer: forward fragments of both phases + W_hhᵀ backward
        fragments, one launch per step."""
        from .lstm import LSTM_SRCS, augmented_codes, model_srcs
        from .pack import KIND_BF16, Packer, make_codes
        if getattr(self, "_pk_model", None) is not model:
            tidx = _t_index("cpu")
            pk = Packer(model_srcs(model))
            pk.add(augmented_codes(self.F, True), self.w_enc, KIND_BF16)
            pk.add(augmented_codes(self.F, False), self.w_dec, KIND_BF16)
            pk.add(make_codes(torch.full_like(tidx, LSTM_SRCS.index("enc_w_hh")), tidx), self.wt_enc, KIND_BF16)
            pk.add(make_codes(torch.full_like(tidx, LSTM_SRCS.index("dec_w_hh")), tidx), self.wt_dec, KIND_BF16)
            self._pk, self._pk_model = pk, model
        return self._pk

    def _scatter_grads(self, model, dwe, dwd, dwo) -> None:
        """GEMM results → ``p.grad`` (views of the DP buckets) in one pack
        launch; the read-out bias gradient is a row sum written in place."""
        from .pack import KIND_F32, Packer, make_codes
        for p in model.parameters():
            if p.grad is None:
                p.grad = torch.zeros_like(p)
        key = (model, tuple(p.grad.data_ptr() for p in model.parameters()))
        if getattr(self, "_gs_key", None) != key:
            F = self.F
            r = torch.arange(4 * H)
            k = torch.arange(H)
            pk = Packer([dwe, dwd, dwo])
            z = lambda n, v: torch.full((n,), v)  # noqa: E731
            pk.add(make_codes(z(4 * H * H, 0), (r[:, None] * KAUG + k[None]).flatten()), model.enc_w_hh.grad.view(-1),
                   KIND_F32)
            pk.add(make_codes(z(4 * H * F, 0), (r[:, None] * KAUG + H + torch.arange(F)[None]).flatten()),
                   model.enc_w_ih.grad.view(-1), KIND_F32)
            pk.add(make_codes(z(4 * H, 0), r * KAUG + BIAS_K), model.enc_b.grad.view(-1), KIND_F32)
            pk.add(make_codes(z(4 * H * H, 1), (r[:, None] * KAUG + k[None]).flatten()), model.dec_w_hh.grad.view(-1),
                   KIND_F32)
            pk.add(make_codes(z(4 * H, 1), r * KAUG + BIAS_K), model.dec_b.grad.view(-1), KIND_F32)
            pk.add(make_codes(z(F * H, 2), torch.arange(F * H)), model.out_w.grad.view(-1), KIND_F32)
            self._gs, self._gs_key = pk, key
        for i, t in enumerate((dwe, dwd, dwo)):
            self._gs.set_src(i, t.contiguous())
        self._gs.run()
        torch.sum(self.dy, 1, out=model.out_b.grad)

    def _pack(self, model) -> None:
        if nat.available():
            self._packer_for(model).run()
            return
        F = self.F
        idx = _frag_index(self.device)
        self.w_enc.copy_(_augment_dev(model.enc_w_hh, model.enc_b, model.enc_w_ih, F).flatten()[idx])
        self.w_dec.copy_(_augment_dev(model.dec_w_hh, model.dec_b, None, F).flatten()[idx])
        tidx = _t_index(self.device)
        self.wt_enc.copy_(model.enc_w_hh.detach().flatten()[tidx])
        self.wt_dec.copy_(model.dec_w_hh.detach().flatten()[tidx])

    phases = 0  # profiling only: restrict the kernel to a subset of its four phases
    batched_gemm = True  # weight-grad reduction as a strided-batched GEMM over time slices

    def pack(self, model) -> None:
        """The weight fragments of the next :meth:`launch` (``launch(..., pack=False)``
        then skips it: a caller can enqueue the packing ahead, e.g. before a stream fork)."""
        self._pack(model)

    def launch(self, model, x: Optional[torch.Tensor], ring: Optional[RingSource] = None,
               pack: bool = True) -> torch.Tensor:
        """Run the fused forward+backward; returns per-window errors ``[B]``.
        ``x [B, T, F]`` windows, or ``ring`` (windows sampled by
        ``win_series``/``win_start``, read straight from the history rings)."""
        lib = nat.require()
        if ring is None:
            _need(x is not None and x.is_cuda and x.dtype == torch.float32 and x.is_contiguous()
                  and tuple(x.shape) == (self.B, self.T, self.F), "x must be contiguous float32 [B, T, F]")
        else:
            _need(ring.win_series is not None, "ring training needs sampled windows (win_series/win_start)")
        _need(model.H == H and model.F == self.F, "model shape mismatch")
        if pack:
            self._pack(model)
        w_out = model.out_w.detach().contiguous()
        b_out = model.out_b.detach().contiguous()
        a = LstmTrainArgs()
        a.x = 0 if x is None else x.data_ptr()
        if ring is not None:
            ring.fill(a.src, self.B, self.F)
        a.B, a.T, a.F = self.B, self.T, self.F
        a.phases = int(self.phases)
        a.w_enc, a.w_dec = self.w_enc.data_ptr(), self.w_dec.data_ptr()
        a.wt_enc, a.wt_dec = self.wt_enc.data_ptr(), self.wt_dec.data_ptr()
        a.w_out, a.b_out = w_out.data_ptr(), b_out.data_ptr()
        a.scratch = self.scratch.data_ptr()
        a.g_enc, a.g_dec = self.g_enc.data_ptr(), self.g_dec.data_ptr()
        a.h_enc, a.h_dec = self.h_enc.data_ptr(), self.h_dec.data_ptr()
        a.dy, a.err = self.dy.data_ptr(), self.err.data_ptr()
        a.loss_scale = 2.0 / (self.B * self.T * self.F)
        a.variant = self.variant
        nat.check(lib.fm_lstm_ae_train(C.byref(a), nat.stream_handle(self.device)), "fm_lstm_ae_train")
        return self.err

    def grads(self, model, x: Optional[torch.Tensor], ring: Optional[RingSource] = None) -> torch.Tensor:
        """Fill ``p.grad`` of every model parameter (overwrite); returns the loss.
        ``x`` may itself be a :class:`RingSource` (the DP trainer passes its
        ``windows`` argument through unchanged)."""
        if isinstance(x, RingSource):
            x, ring = None, x
        self.launch(model, x, ring)
        return self.finish(model)

    def finish(self, model) -> torch.Tensor:
        """Second half of :meth:`grads` (after :meth:`launch`): weight-gradient
        GEMMs + scatter into ``p.grad``.  Split so a caller can enqueue other
        work (the scoring kernel) between the two halves."""
        err = self.err
        F, KB, B, T = self.F, self.T * self.B, self.B, self.T
        if self.batched_gemm:
            dwe = _bmm_sum_f32(self.g_enc, self.h_enc.t(), T)           # [256, 80]
            dwd = _bmm_sum_f32(self.g_dec, self.h_dec[:, :KB].t(), T)   # [256, 80]
        else:
            dwe = _mm_f32(self.g_enc, self.h_enc.t())
            dwd = _mm_f32(self.g_dec, self.h_dec[:, :KB].t())
        # [F, 64]: M = F rows over K = T*B is a GEMV that one GEMM tile cannot spread (58 us as
        # a single hipBLASLt launch at B = 4096); batched over the T slices like dwe / dwd
        if self.batched_gemm:
            dwo = _bmm_sum_f32(self.dy.to(torch.bfloat16), self.h_dec[:H, B:].t(), T)
        else:
            dwo = _mm_f32(self.dy.to(torch.bfloat16), self.h_dec[:H, B:].t())
        if nat.available():
            self._scatter_grads(model, dwe, dwd, dwo)
            return err.mean()
        grads = {
            "enc_w_hh": dwe[:, :H], "enc_w_ih": dwe[:, H:H + F], "enc_b": dwe[:, BIAS_K],
            "dec_w_hh": dwd[:, :H], "dec_b": dwd[:, BIAS_K],
            "out_w": dwo, "out_b": self.dy.sum(1),
        }
        for name, p in model.named_parameters():
            g = grads[name]
            if p.grad is None:
                p.grad = g.detach().clone().view_as(p)
            else:
                p.grad.copy_(g.view_as(p))
        return err.mean()
