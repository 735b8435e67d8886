// Fused K9/K11 detection epilogue shared by the model kernels.
//
// Semantics: foremast_amd/models/detect.py.  Called by every thread of a
// workgroup that owns ONE series after the model has produced a forecast
// function f(h) and a spread sigma for it.
#pragma once
#include "common.h"

#include "args.h"


__device__ __forceinline__ float blk_sum(float v, float* red) {
  v = wave_sum(v);
  __syncthreads();
  if (lane_id() == 0) red[wave_id()] = v;
  __syncthreads();
  float s = 0.f;
  for (int i = 0; i < (int)(blockDim.x / FM_WAVE); ++i) s += red[i];
  __syncthreads();
  return s;
}
__device__ __forceinline__ float blk_max(float v, float* red) {
  v = wave_max(v);
  __syncthreads();
  if (lane_id() == 0) red[wave_id()] = v;
  __syncthreads();
  float s = red[0];
  for (int i = 1; i < (int)(blockDim.x / FM_WAVE); ++i) s = fmaxf(s, red[i]);
  __syncthreads();
  return s;
}

// Same semantics as detect_epilogue below, for a kernel where ONE WAVE owns
// series n (several series per workgroup): lanes stride the columns and the
// reductions are wave-level, so no workgroup barrier is involved.
template <typename ForecastFn>
__device__ __forceinline__ void detect_epilogue_wave(const DetectArgs& d, int n, float sig, float n_valid,
                                                     ForecastFn fcast) {
  if (d.C <= 0) return;
  const int lane = lane_id();
  float thr = d.threshold[n];
  if (d.differs && d.differs[n]) thr *= d.pw_scale;
  const int bnd = d.bound[n];
  const float mlow = d.min_lower[n];
  const bool model_ok = n_valid >= (float)d.min_valid;
  float cnt = 0.f, anyv = 0.f, sc = 0.f;
  for (int c = lane; c < d.C; c += FM_WAVE) {
    const int h = d.horizons[d.h_ld * n + c];
    const float f = fcast(h);
    const float up = f + thr * sig;
    const float lo = fmaxf(f - thr * sig, mlow);
    const long long o = (long long)n * d.C + c;
    if (d.forecast) d.forecast[o] = f;
    if (d.upper) d.upper[o] = up;
    if (d.lower) d.lower[o] = lo;
    if (d.cur) {
      const float x = d.cur[(long long)n * d.ld_cur + c];
      if (x == x) {
        anyv = 1.f;
        const bool an = model_ok && (((bnd & 1) && x > up) || ((bnd & 2) && x < lo));
        cnt += an ? 1.f : 0.f;
        if (an && d.anom_count) {
          const int slot = atomicAdd(d.anom_count, 1);
          if (slot < d.anom_cap) {
            d.anom_series[slot] = n;
            d.anom_col[slot] = c;
            d.anom_val[slot] = x;
          }
        }
        sc = fmaxf(sc, fabsf(x - f) / fmaxf(sig, 1e-12f));
      }
    }
  }
  if (!d.cur) return;
  cnt = wave_sum(cnt);
  anyv = wave_max(anyv);
  sc = wave_max(sc);
  if (lane == 0) {
    const int ic = (int)cnt;
    const int v = ic > 0 ? 1 : ((anyv > 0.f && model_ok) ? 0 : -1);
    d.count[n] = ic;
    d.verdict[n] = (signed char)v;
    d.score[n] = sc;
    if (d.app_id) {
      const int app = d.app_id[n];
      if (v == 1) atomicAdd(&d.app_stats[2 * app], 1);
      if (v >= 0) atomicAdd(&d.app_stats[2 * app + 1], 1);
    }
  }
}

template <typename ForecastFn>
__device__ __forceinline__ void detect_epilogue(const DetectArgs& d, int n, float sig, float n_valid,
                                                ForecastFn fcast, float* red) {
  if (d.C <= 0) return;
  const int tid = threadIdx.x;
  float thr = d.threshold[n];
  if (d.differs && d.differs[n]) thr *= d.pw_scale;
  const int bnd = d.bound[n];
  const float mlow = d.min_lower[n];
  const bool model_ok = n_valid >= (float)d.min_valid;
  float cnt = 0.f, anyv = 0.f, sc = 0.f;
  for (int c = tid; c < d.C; c += blockDim.x) {
    const int h = d.horizons[d.h_ld * n + c];
    const float f = fcast(h);
    const float up = f + thr * sig;
    const float lo = fmaxf(f - thr * sig, mlow);
    const long long o = (long long)n * d.C + c;
    if (d.forecast) d.forecast[o] = f;
    if (d.upper) d.upper[o] = up;
    if (d.lower) d.lower[o] = lo;
    if (d.cur) {
      const float x = d.cur[(long long)n * d.ld_cur + c];
      if (x == x) {
        anyv = 1.f;
        const bool an = model_ok && (((bnd & 1) && x > up) || ((bnd & 2) && x < lo));
        cnt += an ? 1.f : 0.f;
        if (an && d.anom_count) {  // anomalies are rare: one atomic per anomalous point
          const int slot = atomicAdd(d.anom_count, 1);
          if (slot < d.anom_cap) {
            d.anom_series[slot] = n;
            d.anom_col[slot] = c;
            d.anom_val[slot] = x;
          }
        }
        sc = fmaxf(sc, fabsf(x - f) / fmaxf(sig, 1e-12f));
      }
    }
  }
  if (!d.cur) return;
  cnt = blk_sum(cnt, red);
  anyv = blk_max(anyv, red);
  sc = blk_max(sc, red);
  if (tid == 0) {
    const int ic = (int)cnt;
    const int v = ic > 0 ? 1 : ((anyv > 0.f && model_ok) ? 0 : -1);
    d.count[n] = ic;
    d.verdict[n] = (signed char)v;
    d.score[n] = sc;
    if (d.app_id) {
      const int app = d.app_id[n];
      if (v == 1) atomicAdd(&d.app_stats[2 * app], 1);
      if (v >= 0) atomicAdd(&d.app_stats[2 * app + 1], 1);
    }
  }
}
