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

// Per-series thresholds of the detection rules (models/detect.py detect): full
// band (threshold) and, when the canary test says baseline and current differ,
// the lowered band (threshold_low, or threshold * pw_scale) — which only counts
// when at least pw_min_points points fall outside it — and the mean-shift rule
// (shift_thr > 0): the window's mean deviation from the baseline pods' mean, in
// units of the spread s (the one-step sigma with shift_one_step), beyond shift_thr on an
// enabled side.
struct DetThr {
  float full, low, shift, bm;
  bool differs, shift_on;
};
__device__ __forceinline__ DetThr det_thresholds(const DetectArgs& d, int n, int npts) {
  DetThr t;
  t.differs = d.differs && d.differs[n];
  if (d.thr_lut) {  // window-corrected levels of the series' class at its valid-point count
    const int k = npts < d.lut_n ? npts : d.lut_n - 1;
    const float* row = d.thr_lut + (long long)d.thr_cls[n] * 2 * d.lut_n;
    t.full = row[k];
    t.low = row[d.lut_n + k];
  } else {
    t.full = d.threshold[n];
    t.low = d.threshold_low ? d.threshold_low[n] : t.full * d.pw_scale;
  }
  t.shift = d.shift_thr;
  t.bm = (d.base_mean && t.differs) ? d.base_mean[n] : fm_nan();
  t.shift_on = t.differs && d.shift_thr > 0.f && t.bm == t.bm;
  return t;
}

// Pass-1 sums of a series (reduced by the caller)
struct DetSums {
  float cnt_f = 0.f, cnt_l = 0.f, cnt_s = 0.f, zsum = 0.f, nz = 0.f, anyv = 0.f, sc = 0.f;
};

__device__ __forceinline__ bool det_outside(float x, float f, float thr, float s, float mlow, int bnd) {
  return ((bnd & 1) && x > f + thr * s) || ((bnd & 2) && x < fmaxf(f - thr * s, mlow));
}

// Newest window column of series n for the host record (row_out).
__device__ __forceinline__ int det_last_col(const DetectArgs& d, int n) {
  int c = d.tick_min[0] - d.start_min[n];
  return c < 0 ? 0 : (c >= d.last_ncol ? d.last_ncol - 1 : c);
}

// Valid (non-NaN) points of column c, for the threshold table's pre-pass.
__device__ __forceinline__ float det_valid_col(const DetectArgs& d, int n, int c) {
  const float x = d.cur[(long long)n * d.ld_cur + c];
  return x == x ? 1.f : 0.f;
}

// Pass 1 of a column: counts against both bands (the caller reduces them).
template <typename ForecastFn>
__device__ __forceinline__ void det_count_col(const DetectArgs& d, int n, int c, const DetThr& t, float sig, int gidx,
                                              int bnd, float mlow, bool model_ok, ForecastFn& fcast, DetSums& u) {
  const float x = d.cur[(long long)n * d.ld_cur + c];
  if (!(x == x)) return;
  u.anyv = 1.f;
  const int h = d.horizons[d.h_ld * n + c];
  const float f = fcast(h);
  const float s = sig * hstep_factor(d, gidx, h);
  if (model_ok) {
    u.cnt_f += det_outside(x, f, t.full, s, mlow, bnd) ? 1.f : 0.f;
    if (t.differs) u.cnt_l += det_outside(x, f, t.low, s, mlow, bnd) ? 1.f : 0.f;
    if (t.shift_on) {
      const float ss = d.shift_one_step ? sig : s;  // the mean-shift rule's spread
      u.cnt_s += det_outside(x, t.bm, t.shift, ss, mlow, bnd) ? 1.f : 0.f;
      u.zsum += (x - t.bm) / fmaxf(ss, 1e-12f);
      u.nz += 1.f;
    }
  }
  u.sc = fmaxf(u.sc, fabsf(x - f) / fmaxf(s, 1e-12f));
}

// Pass 2 of a column: band of the rule in force (centred on the forecast, or on the
// baseline mean `center` for the mean-shift rule), and the K9 list (rare: one atomic
// per anomalous point of an anomalous series).
template <typename ForecastFn>
__device__ __forceinline__ void det_emit_col(const DetectArgs& d, int n, int c, float thr, float sig, int gidx, int bnd,
                                             float mlow, bool emit, ForecastFn& fcast, float center) {
  const int h = d.horizons[d.h_ld * n + c];
  const float f = fcast(h);
  const bool shifted = center == center;  // the mean-shift rule's band
  const float s = (shifted && d.shift_one_step) ? sig : sig * hstep_factor(d, gidx, h);
  const float fc = shifted ? center : f;
  const float up = fc + thr * s;
  const float lo = fmaxf(fc - thr * s, mlow);
  const long long o = (long long)n * d.C + c;
  if (d.forecast) d.forecast[o] = f;
  if (d.upper) d.upper[o] = up;
  if (d.lower) d.lower[o] = lo;
  if (d.row_out && c == det_last_col(d, n)) {
    d.row_out[4 * (long long)n + 2] = up;
    d.row_out[4 * (long long)n + 3] = lo;
  }
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

// Verdict from the reduced sums; returns the threshold of the rule in force and
// sets *count (anomalous points under that rule) and *center (NaN: the band is
// centred on the forecast).  Precedence: lowered band, full band, mean shift (whose
// band is base_mean +- shift_thr * s).
__device__ __forceinline__ float det_decide(const DetectArgs& d, const DetThr& t, const DetSums& u, int bnd,
                                            int* count, float* center) {
  *center = fm_nan();
  if (t.differs && u.cnt_l >= (float)max(d.pw_min_points, 1)) {
    *count = (int)u.cnt_l;
    return t.low;
  }
  if (u.cnt_f <= 0.f && t.shift_on && u.nz >= (float)max(d.shift_min_points, 1)) {
    const float mz = u.zsum / u.nz;
    if (((bnd & 1) && mz > t.shift) || ((bnd & 2) && mz < -t.shift)) {
      *count = (int)u.cnt_s;
      *center = t.bm;
      return t.shift;
    }
  }
  *count = (int)u.cnt_f;
  return t.full;
}

__device__ __forceinline__ void det_write(const DetectArgs& d, int n, int ic, float anyv, bool model_ok, float sc,
                                          float npts) {
  const int v = ic > 0 ? 1 : ((anyv > 0.f && model_ok) ? 0 : -1);
  d.count[n] = ic;
  d.verdict[n] = (signed char)v;
  d.score[n] = sc;
  if (d.row_out) {
    d.row_out[4 * (long long)n] = (float)v;
    d.row_out[4 * (long long)n + 1] = npts;
  }
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
  float npts = 0.f;
  if (d.cur && (d.thr_lut || d.row_out)) {
    for (int c = lane; c < d.C; c += FM_WAVE) npts += det_valid_col(d, n, c);
    npts = wave_allsum(npts);
  }
  const DetThr t = det_thresholds(d, n, (int)npts);
  const int bnd = d.bound[n];
  const float mlow = d.min_lower[n];
  const bool model_ok = n_valid >= (float)d.min_valid;
  float thr = t.full, center = fm_nan();
  int ic = 0;
  DetSums u;
  if (d.cur) {
    for (int c = lane; c < d.C; c += FM_WAVE) det_count_col(d, n, c, t, sig, gidx, bnd, mlow, model_ok, fcast, u);
    u.cnt_f = wave_allsum(u.cnt_f);
    if (t.differs) u.cnt_l = wave_allsum(u.cnt_l);  // t.differs is wave-uniform (one series per wave)
    if (t.shift_on) {
      u.cnt_s = wave_allsum(u.cnt_s);
      u.zsum = wave_allsum(u.zsum);
      u.nz = wave_allsum(u.nz);
    }
    u.anyv = wave_allmax(u.anyv);
    u.sc = wave_allmax(u.sc);
    thr = det_decide(d, t, u, bnd, &ic, &center);
  }
  const float anyv = u.anyv, sc = u.sc;
  const bool emit = d.anom_count && ic > 0;
  if (d.forecast || d.upper || d.lower || d.row_out || emit)
    for (int c = lane; c < d.C; c += FM_WAVE) det_emit_col(d, n, c, thr, sig, gidx, bnd, mlow, emit, fcast, center);
  if (d.cur && lane == 0) det_write(d, n, ic, anyv, model_ok, sc, npts);
}

// All-reduce over the 16 lanes of a DPP row: quad butterflies, then row rotations by 4
// and 8 (every lane ends with the row's total; rows never mix).
template <bool MAX>
__device__ __forceinline__ float row16_all(float v) {
  auto op = [](float a, float b) { return MAX ? fmaxf(a, b) : a + b; };
  v = op(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xf, 0xf, false)));   // xor 1
  v = op(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xf, 0xf, false)));   // xor 2
  v = op(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x124, 0xf, 0xf, false)));  // row_ror:4
  v = op(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x128, 0xf, 0xf, false)));  // row_ror:8
  return v;
}

// Same semantics as detect_epilogue_wave for kernels where ONE 16-LANE ROW owns series n
// (four series per wave): the deferred epilogues, whose work per series is a window of
// ~10 columns, would leave 54 of 64 lanes idle with a wave per series.  Every branch
// below is uniform over a row (one series), so the row reductions see only active lanes.
template <typename ForecastFn>
__device__ __forceinline__ void detect_epilogue_row(const DetectArgs& d, int n, float sig, float n_valid,
                                                    ForecastFn fcast, int gidx = -1) {
  if (d.C <= 0) return;
  const int gl = lane_id() & 15;
  float npts = 0.f;
  if (d.cur && (d.thr_lut || d.row_out)) {
    for (int c = gl; c < d.C; c += 16) npts += det_valid_col(d, n, c);
    npts = row16_all<false>(npts);
  }
  const DetThr t = det_thresholds(d, n, (int)npts);
  const int bnd = d.bound[n];
  const float mlow = d.min_lower[n];
  const bool model_ok = n_valid >= (float)d.min_valid;
  float thr = t.full, center = fm_nan();
  int ic = 0;
  DetSums u;
  if (d.cur) {
    for (int c = gl; c < d.C; c += 16) det_count_col(d, n, c, t, sig, gidx, bnd, mlow, model_ok, fcast, u);
    u.cnt_f = row16_all<false>(u.cnt_f);
    if (t.differs) u.cnt_l = row16_all<false>(u.cnt_l);
    if (t.shift_on) {
      u.cnt_s = row16_all<false>(u.cnt_s);
      u.zsum = row16_all<false>(u.zsum);
      u.nz = row16_all<false>(u.nz);
    }
    u.anyv = row16_all<true>(u.anyv);
    u.sc = row16_all<true>(u.sc);
    thr = det_decide(d, t, u, bnd, &ic, &center);
  }
  const float anyv = u.anyv, sc = u.sc;
  const bool emit = d.anom_count && ic > 0;
  if (d.forecast || d.upper || d.lower || d.row_out || emit)
    for (int c = gl; c < d.C; c += 16) det_emit_col(d, n, c, thr, sig, gidx, bnd, mlow, emit, fcast, center);
  if (d.cur && gl == 0) det_write(d, n, ic, anyv, model_ok, sc, npts);
}

// One WORKGROUP owns series n: threads stride the columns, block reductions.
template <typename ForecastFn>
__device__ __forceinline__ void detect_epilogue(const DetectArgs& d, int n, float sig, float n_valid,
                                                ForecastFn fcast, float* red, int gidx = -1) {
  if (d.C <= 0) return;
  const int tid = threadIdx.x;
  float npts = 0.f;
  if (d.cur && (d.thr_lut || d.row_out)) {
    for (int c = tid; c < d.C; c += blockDim.x) npts += det_valid_col(d, n, c);
    npts = blk_sum(npts, red);
  }
  const DetThr t = det_thresholds(d, n, (int)npts);
  const int bnd = d.bound[n];
  const float mlow = d.min_lower[n];
  const bool model_ok = n_valid >= (float)d.min_valid;
  float thr = t.full, center = fm_nan();
  int ic = 0;
  DetSums u;
  if (d.cur) {
    for (int c = tid; c < d.C; c += blockDim.x) det_count_col(d, n, c, t, sig, gidx, bnd, mlow, model_ok, fcast, u);
    u.cnt_f = blk_sum(u.cnt_f, red);
    if (t.differs) u.cnt_l = blk_sum(u.cnt_l, red);  // block-uniform: one series per workgroup
    if (t.shift_on) {
      u.cnt_s = blk_sum(u.cnt_s, red);
      u.zsum = blk_sum(u.zsum, red);
      u.nz = blk_sum(u.nz, red);
    }
    u.anyv = blk_max(u.anyv, red);
    u.sc = blk_max(u.sc, red);
    thr = det_decide(d, t, u, bnd, &ic, &center);
  }
  const float anyv = u.anyv, sc = u.sc;
  const bool emit = d.anom_count && ic > 0;
  if (d.forecast || d.upper || d.lower || d.row_out || emit)
    for (int c = tid; c < d.C; c += blockDim.x) det_emit_col(d, n, c, thr, sig, gidx, bnd, mlow, emit, fcast, center);
  if (d.cur && tid == 0) det_write(d, n, ic, anyv, model_ok, sc, npts);
}
