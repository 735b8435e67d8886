// Shared device pieces of the fused LSTM-AE kernels (inference: lstm.hip,
// training: lstm_train.hip): MFMA operand types, activation functions and
// B-fragment packing for v_mfma_f32_32x32x16_bf16 and the CDNA4 block-scaled
// v_mfma_scale_f32_32x32x64_f8f6f4 (e4m3).
#pragma once

#include "common.h"

#include <type_traits>

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// Optional direct read of the model input from the HBM history rings (no
// materialised [N, T, F] window tensor): sample t of window w is ring column
// (start + t) mod R of series row, z-scored with the series' mean / 1/std.
struct LstmRingSrc {
  const void* ring[7];     // per-feature [N, ld] rings (bf16 or fp32); ring[0] == null => dense x
  long long ld;
  int ring_len;
  int bf16;
  int start_col;           // physical column of t = 0 when win_start is null
  int _pad;
  const int* win_series;   // [B] ring row per window (training samples) or null (row = window)
  const int* win_start;    // [B] start column per window (taken mod ring_len) or null
  const float* mean;       // [N, F]
  const float* rstd;       // [N, F]
  const int* head_dev;     // optional device ring head: start columns are then offsets from it
};

namespace fm_lstm {

// per-lane input cursor: dense row pointer, or (ring row, start column)
struct XPos {
  const float* xrow;
  long long row;
  int start;
};

__device__ __forceinline__ XPos make_xpos(const float* x, const LstmRingSrc& s, long long w, int T, int F) {
  XPos p;
  if (!s.ring[0]) {
    p.xrow = x + w * (long long)T * F;
    p.row = w;
    p.start = 0;
  } else {
    p.xrow = nullptr;
    p.row = s.win_series ? s.win_series[w] : w;
    const int off = s.win_start ? s.win_start[w] : s.start_col;
    p.start = ((s.head_dev ? s.head_dev[0] : 0) + off) % s.ring_len;  // any non-negative start
  }
  return p;
}

__device__ __forceinline__ float load_x(const LstmRingSrc& s, const XPos& p, int t, int f, int F) {
  if (p.xrow) return p.xrow[t * F + f];
  int c = p.start + t;
  if (c >= s.ring_len) c -= s.ring_len;
  const long long o = p.row * s.ld + c;
  const float v = s.bf16 ? bf16_to_f32(((const bf16_t*)s.ring[f])[o]) : ((const float*)s.ring[f])[o];
  return (v - s.mean[p.row * F + f]) * s.rstd[p.row * F + f];
}

constexpr int H = 64;
constexpr int TILES = 8;
constexpr int KSTEPS = 5;
constexpr int FRAG_BYTES_BF16 = TILES * KSTEPS * 64 * 16;  // 40 KB
// fp8: CDNA4 block-scaled MFMA, K = 64 per instruction: k-step 0 holds the 64 hidden units
// (each lane half's 32 units in its h-register order), k-step 1 the input and the bias (lane
// half 0, bytes 0..F-1 and 7), so 2 MFMAs per gate tile instead of 5
constexpr int KSTEPS_FP8 = 2;
constexpr int FRAG_BYTES_FP8 = TILES * KSTEPS_FP8 * 64 * 32;    // 32 KB of e4m3
constexpr int SCALE_BYTES_FP8 = TILES * KSTEPS_FP8 * 64;        // E8M0 per (tile, k-step, lane): [lane][16]
                                                                // (lane r + 32 b: k block b of row r)
// h enters the B operand as h * 2^8 (|h| <= 1: e4m3 normals reach down to |h| = 2^-14), scaled
// back by the MFMA (E8M0 127 - 8); inputs and bias enter unscaled (127).  Replicated in all
// four bytes: any op_sel byte reads it.
constexpr int ACT_SHIFT = 8;
constexpr int SCALE_H = 0x77777777;   // 119 = 127 - ACT_SHIFT
constexpr int SCALE_ONE = 0x7f7f7f7f;

// v_exp_f32 (2^x) + v_rcp_f32 (1 ulp): two transcendental issues per
// activation.  (__frcp_rn / '/' lower to the ~10-instruction IEEE division
// sequence.)  Saturates cleanly: exp2 → inf gives rcp → 0.
constexpr float LOG2E = 1.4426950408889634f;
__device__ __forceinline__ float tanh_f(float v) {
  return 2.f * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-2.f * LOG2E * v)) - 1.f;
}

// two fp32 -> packed bf16 (RNE) in ONE v_cvt_pk_bf16_f32 (gfx950); the software
// rounding sequence it replaces cost ~8 VALU + a divergent NaN branch per value,
// 20 % of the scoring kernel's instructions per step
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ bf16_t bf16_hw(float f) {  // one fp32 -> bf16 (RNE), hardware convert
  const __bf16 b = (__bf16)f;
  bf16_t r;
  __builtin_memcpy(&r, &b, 2);
  return r;
}
// the same activations for two units at once: the multiplies / adds become
// packed-FP32 VOP3P ops (v_pk_mul_f32, v_pk_add_f32, v_pk_fma_f32), only the two
// transcendentals per value stay scalar
__device__ __forceinline__ f32x2_t sigm2(f32x2_t v) {
  const f32x2_t t = v * (-LOG2E);
  const f32x2_t d = (f32x2_t){__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)} + 1.f;
  return (f32x2_t){__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
}
__device__ __forceinline__ f32x2_t tanh2(f32x2_t v) {
  const f32x2_t t = v * (-2.f * LOG2E);
  const f32x2_t d = (f32x2_t){__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)} + 1.f;
  const f32x2_t r = (f32x2_t){__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  return r * 2.f - 1.f;
}

__device__ __forceinline__ unsigned pack_bf16x2(float lo, float hi) {
  const bf16x2_t b = __builtin_convertvector((f32x2_t){lo, hi}, bf16x2_t);
  unsigned r;
  __builtin_memcpy(&r, &b, 4);
  return r;
}

__device__ __forceinline__ unsigned pack_fp8x4(float a, float b, float c, float d) {
  int v = 0;
  v = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, v, false);
  v = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, v, true);
  return (unsigned)v;
}

// ---- CDNA4 block-scaled fp8: v_mfma_scale_f32_32x32x64_f8f6f4 (e4m3 A and B) ----------
// lane l holds row (A) / column (B) l & 31 in its 8-VGPR fragment, A and B with the same
// byte <-> k order; measured on the MI355X (scripts/probe_mfma_scale.py, pinned by
// tests/test_lstm.py): bytes 16 b .. 16 b + 15 of lanes r and r + 32 form k block b of
// row r (column c), scaled by 2^(s - 127), s = byte op_sel of lane r + 32 b's (c + 32 b's)
// scale register.
typedef int f8x32 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ f8x32 pack_fp8x32(const float (&v)[32]) {
  f8x32 r;
#pragma unroll
  for (int i = 0; i < 8; ++i) r[i] = (int)pack_fp8x4(v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]);
  return r;
}

// SEL: which byte of the two scale registers holds this MFMA's E8M0 scales (op_sel), so one
// VGPR carries the scales of four k blocks
template <int SEL>
__device__ __forceinline__ f32x16 mfma_scaled(const f8x32& a, const f8x32& b, f32x16 c, int scale_a, int scale_b) {
  // format codes 0 / 0: e4m3 (OCP fp8) for A and B
  return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 0, 0, SEL, scale_a, SEL, scale_b);
}

// bf16 A / B fragment of v_mfma_f32_32x32x16_bf16: 8 x bf16 = uint4
typedef uint4 FragBF16;

__device__ __forceinline__ f32x16 mfma_bf16(const FragBF16& a, const FragBF16& b, f32x16 c) {
  bf16x8_t av, bv;
  __builtin_memcpy(&av, &a, 16);
  __builtin_memcpy(&bv, &b, 16);
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, c, 0, 0, 0);
}

// Model inputs enter the fp8 B operand saturated to the e4m3 range (+-448):
// the conversion would turn an out-of-range z-score -- a regressed series,
// the very thing being detected -- into NaN.  bf16 covers the fp32 range.
__device__ __forceinline__ float sat_fp8(float v) { return fminf(fmaxf(v, -448.f), 448.f); }

// Build the bf16 B fragment for a k-step from 8 fp32 values.
__device__ __forceinline__ FragBF16 make_b_bf16(const float (&v)[8]) {
  FragBF16 r;
  r.x = pack_bf16x2(v[0], v[1]);
  r.y = pack_bf16x2(v[2], v[3]);
  r.z = pack_bf16x2(v[4], v[5]);
  r.w = pack_bf16x2(v[6], v[7]);
  return r;
}

}  // namespace fm_lstm
