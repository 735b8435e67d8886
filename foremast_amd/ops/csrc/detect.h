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

// sigma multiplier of the h-step forecast error of the fitted smoothing model
// (models/detect.py horizon_sigma_factor): with the error-correction updates
// l += a e, b += a b' e, s += g (1 - a) e the h-step error is sum_j c_j e_{T+h-j},
// c_0 = 1, c_j = a (1 + j b') + g (1 - a) [j mod m == 0], so
// v(h) = 1 + a^2 sum_{j<h} (1 + j b')^2 + (seasonal lags) in closed form.
__device__ __forceinline__ float hstep_factor(const DetectArgs& d, int gidx, int h) {
  if (!d.hv_grid || gidx < 0 || h <= 1 || d.hv_mode <= 0) return 1.f;
  const float al = d.hv_grid[3 * gidx];
  const float be = d.hv_mode >= 2 ? d.hv_grid[3 * gidx + 1] : 0.f;
  const float hm1 = (float)(h - 1);
  const float s1 = 0.5f * hm1 * (float)h;
  const float s2 = hm1 * (float)h * (2.f * (float)h - 1.f) * (1.f / 6.f);
  float v = 1.f + al * al * (hm1 + 2.f * be * s1 + be * be * s2);
  if (d.hv_mode == 3 && d.hv_m > 0) {
    const int k = (h - 1) / d.hv_m;
    if (k > 0) {
      const float ga = d.hv_grid[3 * gidx + 2] * (1.f - al), fk = (float)k;
      v += fk * ga * ga + 2.f * ga * al * (fk + (float)d.hv_m * be * 0.5f * fk * (fk + 1.f));
    }
  }
  return sqrtf(v);
}

// Per-series thresholds of the two detection rules (models/detect.py detect):
// full band (threshold) and, when the canary test says baseline and current
// differ, the lowered band (threshold_low, or threshold * pw_scale) — which only
// counts when at least pw_min_points points fall outside it.
struct DetThr {
  float full, low;
  bool differs;
};
__device__ __forceinline__ DetThr det_thresholds(const DetectArgs& d, int n) {
  DetThr t;
  t.full = d.threshold[n];
  t.differs = d.differs && d.differs[n];
  t.low = d.threshold_low ? d.threshold_low[n] : t.full * d.pw_scale;
  return t;
}

__device__ __forceinline__ bool det_outside(float x, float f, float thr, float s, float mlow, int bnd) {
  return ((bnd & 1) && x > f + thr * s) || ((bnd & 2) && x < fmaxf(f - thr * s, mlow));
}

// Pass 1 of a column: counts against both bands (the caller reduces them).
template <typename ForecastFn>
__device__ __forceinline__ void det_count_col(const DetectArgs& d, int n, int c, const DetThr& t, float sig, int gidx,
                                              int bnd, float mlow, bool model_ok, ForecastFn& fcast, float& cnt_f,
                                              float& cnt_l, float& anyv, float& sc) {
  const float x = d.cur[(long long)n * d.ld_cur + c];
  if (!(x == x)) return;
  anyv = 1.f;
  const int h = d.horizons[d.h_ld * n + c];
  const float f = fcast(h);
  const float s = sig * hstep_factor(d, gidx, h);
  if (model_ok) {
    cnt_f += det_outside(x, f, t.full, s, mlow, bnd) ? 1.f : 0.f;
    if (t.differs) cnt_l += det_outside(x, f, t.low, s, mlow, bnd) ? 1.f : 0.f;
  }
  sc = fmaxf(sc, fabsf(x - f) / fmaxf(s, 1e-12f));
}

// Pass 2 of a column: band of the rule in force, and the K9 list (rare: one atomic
// per anomalous point of an anomalous series).
template <typename ForecastFn>
__device__ __forceinline__ void det_emit_col(const DetectArgs& d, int n, int c, float thr, float sig, int gidx, int bnd,
                                             float mlow, bool emit, ForecastFn& fcast) {
  const int h = d.horizons[d.h_ld * n + c];
  const float f = fcast(h);
  const float s = sig * hstep_factor(d, gidx, h);
  const float up = f + thr * s;
  const float lo = fmaxf(f - thr * s, mlow);
  const long long o = (long long)n * d.C + c;
  if (d.forecast) d.forecast[o] = f;
  if (d.upper) d.upper[o] = up;
  if (d.lower) d.lower[o] = lo;
  if (emit) {
    const float x = d.cur[(long long)n * d.ld_cur + c];
    if (x == x && (((bnd & 1) && x > up) || ((bnd & 2) && x < lo))) {
      const int slot = atomicAdd(d.anom_count, 1);
      if (slot < d.anom_cap) {
        d.anom_series[slot] = n;
        d.anom_col[slot] = c;
        d.anom_val[slot] = x;
      }
    }
  }
}

// Verdict from the reduced counts; returns the threshold of the rule in force and
// sets *count (anomalous points under that rule).
__device__ __forceinline__ float det_decide(const DetectArgs& d, const DetThr& t, float cnt_f, float cnt_l, int* count) {
  const bool low_rule = t.differs && cnt_l >= (float)max(d.pw_min_points, 1);
  *count = (int)(low_rule ? cnt_l : cnt_f);
  return low_rule ? t.low : t.full;
}

__device__ __forceinline__ void det_write(const DetectArgs& d, int n, int ic, float anyv, bool model_ok, float sc) {
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

// Same semantics as detect_epilogue below, for a kernel where ONE WAVE owns
// series n (several series per workgroup): lanes stride the columns and the
// reductions are wave-level, so no workgroup barrier is involved.  gidx: grid
// index of the fitted smoothing parameters (horizon variance), -1 for none.
template <typename ForecastFn>
__device__ __forceinline__ void detect_epilogue_wave(const DetectArgs& d, int n, float sig, float n_valid,
                                                     ForecastFn fcast, int gidx = -1) {
  if (d.C <= 0) return;
  const int lane = lane_id();
  const DetThr t = det_thresholds(d, n);
  const int bnd = d.bound[n];
  const float mlow = d.min_lower[n];
  const bool model_ok = n_valid >= (float)d.min_valid;
  float thr = t.full;
  int ic = 0;
  float anyv = 0.f, sc = 0.f;
  if (d.cur) {
    float cnt_f = 0.f, cnt_l = 0.f;
    for (int c = lane; c < d.C; c += FM_WAVE)
      det_count_col(d, n, c, t, sig, gidx, bnd, mlow, model_ok, fcast, cnt_f, cnt_l, anyv, sc);
    cnt_f = wave_allsum(cnt_f);
    cnt_l = t.differs ? wave_allsum(cnt_l) : 0.f;  // t.differs is wave-uniform (one series per wave)
    anyv = wave_allmax(anyv);
    sc = wave_allmax(sc);
    thr = det_decide(d, t, cnt_f, cnt_l, &ic);
  }
  const bool emit = d.anom_count && ic > 0;
  if (d.forecast || d.upper || d.lower || emit)
    for (int c = lane; c < d.C; c += FM_WAVE) det_emit_col(d, n, c, thr, sig, gidx, bnd, mlow, emit, fcast);
  if (d.cur && lane == 0) det_write(d, n, ic, anyv, model_ok, sc);
}

// One WORKGROUP owns series n: threads stride the columns, block reductions.
template <typename ForecastFn>
__device__ __forceinline__ void detect_epilogue(const DetectArgs& d, int n, float sig, float n_valid,
                                                ForecastFn fcast, float* red, int gidx = -1) {
  if (d.C <= 0) return;
  const int tid = threadIdx.x;
  const DetThr t = det_thresholds(d, n);
  const int bnd = d.bound[n];
  const float mlow = d.min_lower[n];
  const bool model_ok = n_valid >= (float)d.min_valid;
  float thr = t.full;
  int ic = 0;
  float anyv = 0.f, sc = 0.f;
  if (d.cur) {
    float cnt_f = 0.f, cnt_l = 0.f;
    for (int c = tid; c < d.C; c += blockDim.x)
      det_count_col(d, n, c, t, sig, gidx, bnd, mlow, model_ok, fcast, cnt_f, cnt_l, anyv, sc);
    cnt_f = blk_sum(cnt_f, red);
    cnt_l = blk_sum(cnt_l, red);
    anyv = blk_max(anyv, red);
    sc = blk_max(sc, red);
    thr = det_decide(d, t, cnt_f, cnt_l, &ic);
  }
  const bool emit = d.anom_count && ic > 0;
  if (d.forecast || d.upper || d.lower || emit)
    for (int c = tid; c < d.C; c += blockDim.x) det_emit_col(d, n, c, thr, sig, gidx, bnd, mlow, emit, fcast);
  if (d.cur && tid == 0) det_write(d, n, ic, anyv, model_ok, sc);
}
