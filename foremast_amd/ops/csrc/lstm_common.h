// Shared device pieces of the fused LSTM-AE kernels (inference: lstm.hip,
// training: lstm_train.hip): MFMA operand types, activation functions and
// B-fragment packing for v_mfma_f32_32x32x16_{bf16,fp8}.
#pragma once

#include "common.h"

#include <type_traits>

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace fm_lstm {
constexpr int H = 64;
constexpr int TILES = 8;
constexpr int KSTEPS = 5;
constexpr int FRAG_BYTES_BF16 = TILES * KSTEPS * 64 * 16;  // 40 KB
constexpr int FRAG_BYTES_FP8 = TILES * KSTEPS * 64 * 8;    // 20 KB

// v_exp_f32 (2^x) + v_rcp_f32 (1 ulp): two transcendental issues per
// activation.  (__frcp_rn / '/' lower to the ~10-instruction IEEE division
// sequence.)  Saturates cleanly: exp2 → inf gives rcp → 0.
constexpr float LOG2E = 1.4426950408889634f;
__device__ __forceinline__ float sigm(float v) {
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-LOG2E * v));
}
__device__ __forceinline__ float tanh_f(float v) {
  return 2.f * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-2.f * LOG2E * v)) - 1.f;
}

__device__ __forceinline__ unsigned pack_bf16x2(float lo, float hi) {
  return (unsigned)f32_to_bf16(lo) | ((unsigned)f32_to_bf16(hi) << 16);
}

__device__ __forceinline__ unsigned pack_fp8x4(float a, float b, float c, float d) {
  int v = 0;
  v = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, v, false);
  v = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, v, true);
  return (unsigned)v;
}

template <bool FP8>
struct Frag {
  // bf16: 8 x bf16 = uint4; fp8: 8 x fp8 = uint2
  typedef typename std::conditional<FP8, uint2, uint4>::type T;
};

template <bool FP8>
__device__ __forceinline__ f32x16 mfma(const typename Frag<FP8>::T& a, const typename Frag<FP8>::T& b, f32x16 c) {
  if constexpr (FP8) {
    long av, bv;
    __builtin_memcpy(&av, &a, 8);
    __builtin_memcpy(&bv, &b, 8);
    return __builtin_amdgcn_mfma_f32_32x32x16_fp8_fp8(av, bv, c, 0, 0, 0);
  } else {
    bf16x8_t av, bv;
    __builtin_memcpy(&av, &a, 16);
    __builtin_memcpy(&bv, &b, 16);
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, c, 0, 0, 0);
  }
}

// Build the B fragment for a k-step from 8 fp32 values (already scaled).
template <bool FP8>
__device__ __forceinline__ typename Frag<FP8>::T make_b(const float (&v)[8]) {
  typename Frag<FP8>::T r;
  if constexpr (FP8) {
    r.x = pack_fp8x4(v[0], v[1], v[2], v[3]);
    r.y = pack_fp8x4(v[4], v[5], v[6], v[7]);
  } else {
    r.x = pack_bf16x2(v[0], v[1]);
    r.y = pack_bf16x2(v[2], v[3]);
    r.z = pack_bf16x2(v[4], v[5]);
    r.w = pack_bf16x2(v[6], v[7]);
  }
  return r;
}

}  // namespace fm_lstm
