// Shared device helpers for the foremast gfx950 (CDNA4) kernels.
//
// Wave size is 64 on CDNA; every cross-lane idiom here is written for 64
// lanes (`__shfl*` width 64, 64-bit ballots).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define FM_WAVE 64

typedef float v2f __attribute__((ext_vector_type(2)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef unsigned short bf16_t;  // raw bf16 bits (torch.bfloat16 storage)

__device__ __forceinline__ float bf16_to_f32(bf16_t v) {
  return __uint_as_float(((unsigned)v) << 16);
}

__device__ __forceinline__ bf16_t f32_to_bf16(float f) {
  unsigned u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x007fffffu)) return (bf16_t)((u >> 16) | 0x40);
  unsigned r = 0x7fffu + ((u >> 16) & 1u);  // round to nearest even
  return (bf16_t)((u + r) >> 16);
}

template <typename T> __device__ __forceinline__ float to_f32(T v);
template <> __device__ __forceinline__ float to_f32<float>(float v) { return v; }
template <> __device__ __forceinline__ float to_f32<bf16_t>(bf16_t v) { return bf16_to_f32(v); }

template <typename T> __device__ __forceinline__ T from_f32(float v);
template <> __device__ __forceinline__ float from_f32<float>(float v) { return v; }
template <> __device__ __forceinline__ bf16_t from_f32<bf16_t>(float v) { return f32_to_bf16(v); }

__device__ __forceinline__ int lane_id() { return threadIdx.x & (FM_WAVE - 1); }
__device__ __forceinline__ int wave_id() { return threadIdx.x / FM_WAVE; }

__device__ __forceinline__ float fm_nan() { return __uint_as_float(0x7fc00000u); }

// ---- wave (64-lane) reductions -------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, FM_WAVE);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, FM_WAVE));
  return v;
}
__device__ __forceinline__ v2f wave_sum2(v2f v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    v.x += __shfl_xor(v.x, o, FM_WAVE);
    v.y += __shfl_xor(v.y, o, FM_WAVE);
  }
  return v;
}

// All-lane reductions with DPP row scans + row broadcasts (no LDS permute round trips);
// the result is read from lane 63 as a wave-uniform value.  Every lane must be active.
template <int CTRL, int RM, bool BC>
__device__ __forceinline__ float dpp_f(float old, float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(v), CTRL, RM, 0xf, BC));
}
__device__ __forceinline__ float wave_allsum(float v) {
  v += dpp_f<0x111, 0xf, false>(0.f, v);  // row_shr:1..8 (lanes without a source add 0)
  v += dpp_f<0x112, 0xf, false>(0.f, v);
  v += dpp_f<0x114, 0xf, false>(0.f, v);
  v += dpp_f<0x118, 0xf, false>(0.f, v);
  v += dpp_f<0x142, 0xa, false>(0.f, v);  // row_bcast:15 -> rows 1, 3
  v += dpp_f<0x143, 0xc, false>(0.f, v);  // row_bcast:31 -> rows 2, 3
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), FM_WAVE - 1));
}
template <int CTRL, int RM>
__device__ __forceinline__ int dpp_i(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, RM, 0xf, false);
}
// integer all-lane sum (exact; the same DPP pattern as wave_allsum)
__device__ __forceinline__ int wave_allsum_i(int v) {
  v += dpp_i<0x111, 0xf>(v);
  v += dpp_i<0x112, 0xf>(v);
  v += dpp_i<0x114, 0xf>(v);
  v += dpp_i<0x118, 0xf>(v);
  v += dpp_i<0x142, 0xa>(v);
  v += dpp_i<0x143, 0xc>(v);
  return __builtin_amdgcn_readlane(v, FM_WAVE - 1);
}
__device__ __forceinline__ float wave_allmax(float v) {
  const float lo = -__builtin_huge_valf();
  v = fmaxf(v, dpp_f<0x111, 0xf, false>(lo, v));
  v = fmaxf(v, dpp_f<0x112, 0xf, false>(lo, v));
  v = fmaxf(v, dpp_f<0x114, 0xf, false>(lo, v));
  v = fmaxf(v, dpp_f<0x118, 0xf, false>(lo, v));
  v = fmaxf(v, dpp_f<0x142, 0xa, false>(lo, v));
  v = fmaxf(v, dpp_f<0x143, 0xc, false>(lo, v));
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), FM_WAVE - 1));
}

__device__ __forceinline__ v2f shfl_up2(v2f v, int d) {
  v2f r;
  r.x = __shfl_up(v.x, d, FM_WAVE);
  r.y = __shfl_up(v.y, d, FM_WAVE);
  return r;
}
__device__ __forceinline__ v2f shfl2(v2f v, int src) {
  v2f r;
  r.x = __shfl(v.x, src, FM_WAVE);
  r.y = __shfl(v.y, src, FM_WAVE);
  return r;
}

__device__ __forceinline__ v2f splat2(float a) { v2f r; r.x = a; r.y = a; return r; }

// erfc-based normal survival function and chi^2(1) survival.
__device__ __forceinline__ float norm_sf(float z) { return 0.5f * erfcf(z * 0.70710678118654752f); }

#define FM_CHECK_LAUNCH() (hipGetLastError())
