"""Table-driven weight packing for the LSTM kernels (``csrc/pack.hip``).

Every training step changes the LSTM-AE parameters, and both MFMA kernels
want them in their own fragment orders (scoring: augmented ``[W_hh | W_ih |
b]`` A fragments in bf16 or fp8; training: the same plus ``W_hhᵀ`` backward
fragments).  Doing that with torch index/convert ops costs ~15 launches per
step, each longer on the host than on the GPU.  Here every output element is
described by one int32 *code* (which parameter, which offset, which
multiplier class) built once from the reference index maps, and one native
launch produces every segment.  fp8 segments are block-scaled for the CDNA4
``v_mfma_scale_f32_32x32x64_f8f6f4``: each 32-value k block of an A-fragment row
shares an E8M0 scale, the smallest power of two that brings its absolute maximum
within e4m3's 448 (:func:`e8m0_blocks`, :func:`fp8_blocks_lane_major`).

:func:`reference_gather` evaluates the same codes with torch (CPU tests and
the non-GPU path).
"""

from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import torch

from . import _native as nat

SRC_BITS, CLS_BITS = 26, 24
KIND_F32, KIND_BF16, KIND_FP8 = 0, 1, 2


class PackSeg(C.Structure):
    _fields_ = [("code", C.c_void_p), ("out", C.c_void_p), ("n", C.c_int), ("kind", C.c_int),
                ("mul", C.c_float * 4)]


class PackArgs(C.Structure):
    _fields_ = [("src", C.c_void_p * 8), ("seg", PackSeg * 8), ("nseg", C.c_int), ("_pad", C.c_int)]


FP8_CHUNK = 32   # e4m3 bytes one lane holds per MFMA k-step (v_mfma_scale_f32_32x32x64_f8f6f4: K = 64)
FP8_LANES = 64   # scales are stored lane-major: step s of lane l at (l * steps + s)


def e8m0_blocks(v: torch.Tensor):
    """Block-scaled e4m3 of ``v [blocks, k]``: (codes uint8 ``[blocks, k]``, E8M0
    uint8 ``[blocks]``).  The block exponent e is the smallest integer with
    ``absmax <= 448 * 2^e`` (from the exact frexp of absmax, as csrc/pack.hip
    computes it), the codes are ``v * 2^-e`` rounded to e4m3, the scale byte
    ``e + 127``; an all-zero block gets e = 0."""
    v = v.float()
    amax = v.abs().amax(1)
    m, x = torch.frexp(amax)
    e = torch.where(amax > 0, x - 9 + (m > 0.875).to(x.dtype), torch.zeros_like(x)).clamp(-127, 127)
    q = torch.ldexp(v, -e[:, None].to(v.dtype)).to(torch.float8_e4m3fn).view(torch.uint8)
    return q, (e + 127).to(torch.uint8)


def fp8_blocks_lane_major(v: torch.Tensor) -> torch.Tensor:
    """A block-scaled fp8 segment of the values ``v`` (logical MFMA A fragments
    ``[steps, 64 lanes, 32 bytes]``), stored half-major ``[steps, 2 halves, 64 lanes, 16
    bytes]`` so the kernel's 16-byte LDS reads are lane-contiguous (no bank conflicts),
    then the scales lane-major.  Measured on
    the MI355X (``scripts/probe_mfma_scale.py``): bytes 16 b .. 16 b + 15 of lanes r
    AND r + 32 form one 32-value k block of row r, scaled by the byte in lane r + 32 b's
    scale register; so each block's E8M0 is stored in lane r + 32 b."""
    steps = v.numel() // (FP8_LANES * FP8_CHUNK)
    g = v.reshape(steps, 2, 32, 2, 16).permute(0, 2, 3, 1, 4).reshape(steps * 64, 32)   # [(step, r, b), (h, j)]
    q, sc = e8m0_blocks(g)
    q = q.view(steps, 32, 2, 2, 16).permute(0, 2, 3, 1, 4).reshape(-1)                 # [step, b, h, r, j]
    lane_sc = sc.view(steps, 32, 2).permute(0, 2, 1).reshape(steps, FP8_LANES)         # lane = r + 32 b
    return torch.cat([q, lane_sc.t().reshape(-1)])


def fp8_segment_bytes(n: int) -> int:
    """Bytes of a block-scaled fp8 segment of n codes: the codes, then one scale byte per
    (k-step, lane)."""
    return n + n // FP8_CHUNK


nat.register("fm_pack", [C.POINTER(PackArgs), C.c_void_p])
nat.register("fm_pack_args_size", [], C.c_longlong)


def make_codes(src: torch.Tensor, off: torch.Tensor, cls: Optional[torch.Tensor] = None,
               valid: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Encode (source id, offset, multiplier class) per output element."""
    off = off.long()
    if off.numel() and int(off.max()) >= 1 << CLS_BITS:
        raise ValueError("pack offset exceeds 24 bits")
    c = (src.long() << SRC_BITS) | off
    if cls is not None:
        c = c | (cls.long() << CLS_BITS)
    if valid is not None:
        c = torch.where(valid, c, torch.full_like(c, -1))
    return c.to(torch.int32)


def reference_gather(code: torch.Tensor, srcs: Sequence[torch.Tensor], mul=(1.0, 1.0, 1.0, 1.0)) -> torch.Tensor:
    """fp32 value of every coded element (the kernel before conversion)."""
    c = code.long().cpu()
    out = torch.zeros(c.numel(), dtype=torch.float32)
    ok = c >= 0
    sid = (c >> SRC_BITS) & 7
    cls = (c >> CLS_BITS) & 3
    off = c & ((1 << CLS_BITS) - 1)
    m = torch.tensor(list(mul), dtype=torch.float32)
    for s, t in enumerate(srcs):
        sel = ok & (sid == s)
        if sel.any():
            out[sel] = t.detach().float().cpu().flatten()[off[sel]] * m[cls[sel]]
    return out


@dataclass
class _Seg:
    code: torch.Tensor
    out: torch.Tensor
    kind: int
    mul: tuple = (1.0, 1.0, 1.0, 1.0)


@dataclass
class Packer:
    """A fixed set of segments over a fixed list of source tensors; the
    ctypes argument block is built once, so :meth:`run` costs one C call."""
    srcs: List[torch.Tensor]
    segs: List[_Seg] = field(default_factory=list)
    _args: Optional[PackArgs] = None

    def add(self, code: torch.Tensor, out: torch.Tensor, kind: int, mul=(1.0, 1.0, 1.0, 1.0)) -> "Packer":
        if len(self.segs) == 8:
            raise ValueError("at most 8 pack segments")
        n = code.numel()
        if kind == KIND_FP8 and n % (FP8_CHUNK * FP8_LANES):
            raise ValueError(f"an fp8 segment holds whole k-steps of {FP8_LANES} x {FP8_CHUNK} A-fragment bytes")
        want_n = fp8_segment_bytes(n) if kind == KIND_FP8 else n
        if out.numel() != want_n or not out.is_contiguous():
            raise ValueError("pack output must be contiguous with one element per code (fp8: plus the scales)")
        want = {KIND_F32: torch.float32, KIND_BF16: torch.bfloat16, KIND_FP8: torch.uint8}[kind]
        if out.dtype != want:
            raise ValueError(f"pack kind {kind} writes {want}, got {out.dtype}")
        self.segs.append(_Seg(code.to(out.device, torch.int32).contiguous(), out, kind, tuple(mul)))
        self._args = None
        return self

    def set_src(self, i: int, t: torch.Tensor) -> None:
        """Re-point source ``i`` (e.g. a freshly allocated GEMM output)."""
        self.srcs[i] = t
        if self._args is not None:
            self._args.src[i] = t.data_ptr()

    def _build(self) -> PackArgs:
        a = PackArgs()
        if len(self.srcs) > 8:
            raise ValueError("at most 8 pack sources")
        for i, t in enumerate(self.srcs):
            if t.dtype != torch.float32 or not t.is_contiguous():
                raise ValueError("pack sources must be contiguous float32")
            a.src[i] = t.data_ptr()
        for i, s in enumerate(self.segs):
            a.seg[i].code, a.seg[i].out = s.code.data_ptr(), s.out.data_ptr()
            a.seg[i].n, a.seg[i].kind = s.code.numel(), s.kind
            for j in range(4):
                a.seg[i].mul[j] = s.mul[j]
        a.nseg = len(self.segs)
        return a

    def run(self) -> None:
        if self._args is None:
            self._args = self._build()
        nat.check(nat.require().fm_pack(C.byref(self._args), nat.stream_handle(self.segs[0].out.device)), "fm_pack")

    def run_reference(self) -> None:
        """Same outputs with torch ops (CPU / no native library)."""
        for i, s in enumerate(self.segs):
            v = reference_gather(s.code, self.srcs, s.mul).to(s.out.device)
            if s.kind == KIND_F32:
                s.out.copy_(v)
            elif s.kind == KIND_BF16:
                s.out.copy_(v.to(torch.bfloat16))
            else:
                s.out.copy_(fp8_blocks_lane_major(v))
