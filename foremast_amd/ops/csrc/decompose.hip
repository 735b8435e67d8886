// K4: classical additive seasonal decomposition (trend / seasonal / resid)
// of every series of a history ring, one workgroup per series.
//
// Semantics: foremast_amd/models/decompose.py (NaN-aware 2 x m centred MA
// trend, centred per-phase means of the detrended series, residual).
//
// Schedule (512 threads, the series read from HBM exactly once):
//  0. coalesced staging of the ring window (all of a thread's loads in flight
//     at once, samples kept in registers) into LDS as fp32 (+ block mean of
//     the valid values: the offset that keeps the fp32 prefix sums small —
//     the MA is a difference of two prefix sums);
//  1. exclusive prefix sums of valid*(y - mean) (in place over the staged
//     copy) and of the valid count (uint16), per-thread contiguous chunks +
//     one shuffle scan + one LDS round;
//  2. trend per sample from the prefix sums (O(1) each), kept in registers;
//     the detrended series overwrites the prefix array;
//  3. per phase p (strided over threads): mean over periods of y - trend;
//  4. one coalesced output pass: seasonal = phase_mean[t mod m], resid (the
//     trend is stored in pass 2).  LDS: 6 (T+1) + 4 m bytes (66 KiB at T = 10080, m = 1440), so
//     two workgroups share a CU.
//
// Scoring mode (det.C > 0, the ML_ALGORITHM=seasonal_decompose scorer): the residual RMS
// is reduced in pass 4 and the forecast f(h) = trend_e + slope (T - 1 + h - t_e) +
// seasonal[(T - 1 + h) mod m] (t_e: the last sample with a centred-MA trend, slope over
// the last season of trend) runs through the shared band / verdict epilogue (detect.h);
// with the full outputs null, a series costs one HBM read and no [N, T] writes.
#include "common.h"
#include "args.h"
#include "detect.h"

struct DecompArgs {
  const void* hist;   // [N, ld] ring (bf16 or fp32)
  long long ld;
  int ring_len;
  int head;
  int T;              // samples (logical order from head)
  int N;
  int m;              // period
  int bf16;
  float* trend;       // [N, T] or null
  float* seasonal;    // [N, T] or null
  float* resid;       // [N, T] or null
  float* phase_means; // [N, m] or null
  // scoring mode (det.C > 0): forecast parameters, residual RMS, valid count
  float* fc_level;    // [N] trend at t_e (NaN: no trend defined) or null
  float* fc_slope;    // [N] trend slope per step or null
  float* sigma;       // [N] residual RMS or null
  float* nvalid;      // [N] valid samples or null
  DetectArgs det;
};

extern __shared__ __attribute__((aligned(16))) char fm_dec_smem[];

namespace {

constexpr int BLOCK = 512;
constexpr int MAX_ITEMS = 32;  // samples per thread held in registers: T <= 16384

template <typename TIN>
__device__ __forceinline__ float load_y(const DecompArgs& a, const TIN* row, int i) {
  int c = a.head + i;
  if (c >= a.ring_len) c -= a.ring_len;
  return to_f32<TIN>(row[c]);
}

__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x / FM_WAVE;
  __syncthreads();
  if (lane_id() == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < BLOCK / FM_WAVE; ++i) s += red[i];
  return s;
}

// exclusive block scan of one value per thread
__device__ __forceinline__ v2f block_exscan2(v2f v, float* red) {
  const int lane = lane_id(), w = threadIdx.x / FM_WAVE;
  v2f inc = v;
#pragma unroll
  for (int o = 1; o < FM_WAVE; o <<= 1) {
    const v2f t = shfl_up2(inc, o);
    if (lane >= o) inc += t;
  }
  __syncthreads();
  if (lane == FM_WAVE - 1) {
    red[2 * w] = inc.x;
    red[2 * w + 1] = inc.y;
  }
  __syncthreads();
  v2f off = {0.f, 0.f};
  for (int i = 0; i < w; ++i) {
    off.x += red[2 * i];
    off.y += red[2 * i + 1];
  }
  return off + inc - v;
}

template <typename TIN>
__global__ __launch_bounds__(BLOCK) void decompose_kernel(const DecompArgs a) {
  const int n = blockIdx.x;
  const TIN* row = (const TIN*)a.hist + (long long)n * a.ld;
  const int T = a.T, m = a.m, tid = threadIdx.x;
  float* S = (float*)fm_dec_smem;    // [T+1] staged series, then (in place) prefix of valid*(y - ybar)
  float* pm = S + (T + 1);           // [m]
  float* red = pm + m;               // [2 * waves]
  unsigned short* Cn = (unsigned short*)(red + 2 * (BLOCK / FM_WAVE));  // [T+1] prefix of valid (exact: T < 2^16)

  // 0. stage (coalesced) + mean of valid values.  All loads of a thread are issued back
  //    to back (clamped index, no per-element branch) and the samples stay in registers
  //    for the detrended series.
  float yr[MAX_ITEMS];
#pragma unroll
  for (int k = 0; k < MAX_ITEMS; ++k)
    if (k * BLOCK < T) yr[k] = load_y<TIN>(a, row, min(tid + k * BLOCK, T - 1));
  float sv = 0.f, cv = 0.f;
#pragma unroll
  for (int k = 0; k < MAX_ITEMS; ++k) {
    const int t = tid + k * BLOCK;
    if (t < T) {
      const float y = yr[k];
      S[t] = y;
      if (y == y) { sv += y; cv += 1.f; }
    }
  }
  const float ssum = block_sum(sv, red);
  const float csum = block_sum(cv, red);
  const float ybar = csum > 0.f ? ssum / csum : 0.f;

  // 1. prefix sums, contiguous chunk per thread (reads the staged copy and overwrites it
  //    with the prefix: every thread only touches its own chunk)
  const int chunk = (T + BLOCK - 1) / BLOCK;
  const int i0 = min(T, tid * chunk), i1 = min(T, i0 + chunk);
  v2f loc = {0.f, 0.f};
  for (int i = i0; i < i1; ++i) {
    const float y = S[i];
    if (y == y) { loc.x += y - ybar; loc.y += 1.f; }
  }
  v2f run = block_exscan2(loc, red);
  for (int i = i0; i < i1; ++i) {
    const float y = S[i];
    S[i] = run.x;
    Cn[i] = (unsigned short)run.y;
    if (y == y) { run.x += y - ybar; run.y += 1.f; }
  }
  if (i1 == T && i0 < i1) { S[T] = run.x; Cn[T] = (unsigned short)run.y; }
  __syncthreads();

  const int h = m / 2;
  const bool even = (m & 1) == 0;
  const float inv_m = 1.f / (float)m;
  // trend at t (NaN at the edges / when < half the window is valid)
  auto trend_at = [&](int t) -> float {
    if (t < h || t + h > T - 1) return fm_nan();
    float num, den;
    auto cn = [&](int i) { return (float)Cn[i]; };
    if (even) {
      num = (S[t + h] - S[t - h + 1]);
      den = (cn(t + h) - cn(t - h + 1));
      const float ca = cn(t - h + 1) - cn(t - h), cb = cn(t + h + 1) - cn(t + h);
      num += 0.5f * ((S[t - h + 1] - S[t - h]) + (S[t + h + 1] - S[t + h]));
      den += 0.5f * (ca + cb);
    } else {
      num = S[t + h + 1] - S[t - h];
      den = cn(t + h + 1) - cn(t - h);
    }
    num *= inv_m;
    den *= inv_m;
    return den >= 0.5f ? ybar + num * __builtin_amdgcn_rcpf(den) : fm_nan();  // den >= 0.5: rcp is 1 ulp
  };

  // 2. trend once per sample into registers (t = tid + k*BLOCK); after a
  //    barrier S is free and becomes the detrended series D
  //    (the trend output is stored here, so its 4 bytes per sample leave while the
  //    workgroup still has the phase-mean pass to do)
  const long long base = (long long)n * T;
  float tr_r[MAX_ITEMS];
#pragma unroll
  for (int k = 0; k < MAX_ITEMS; ++k) {
    const int t = tid + k * BLOCK;
    tr_r[k] = t < T ? trend_at(t) : 0.f;
    if (t < T && a.trend) a.trend[base + t] = tr_r[k];
  }
  // scoring mode: the last defined trend and the one a season earlier (every thread, from
  // the prefix sums, before they are overwritten)
  const int te = T - 1 - h;
  const float tr_e = trend_at(te), tr_p = te - m >= 0 ? trend_at(te - m) : fm_nan();
  __syncthreads();
  float* D = S;
#pragma unroll
  for (int k = 0; k < MAX_ITEMS; ++k) {
    const int t = tid + k * BLOCK;
    if (t < T) D[t] = yr[k] - tr_r[k];
  }
  __syncthreads();

  // 3. phase means of the detrended series
  for (int p = tid; p < m; p += BLOCK) {
    float s = 0.f, c = 0.f;
    for (int t = p; t < T; t += m) {
      const float d = D[t];
      if (d == d) { s += d; c += 1.f; }
    }
    pm[p] = c > 0.f ? s / c : 0.f;
  }
  __syncthreads();
  float ps = 0.f;
  for (int p = tid; p < m; p += BLOCK) ps += pm[p];
  const float pmean = block_sum(ps, red) / (float)m;
  for (int p = tid; p < m; p += BLOCK) {
    pm[p] -= pmean;
    if (a.phase_means) a.phase_means[(long long)n * m + p] = pm[p];
  }
  __syncthreads();

  // 4. outputs (coalesced) and the residual sum of squares
  const int pstep = BLOCK % m;  // phase of t = tid + k*BLOCK, advanced without an integer division per sample
  int ph = tid % m;
  float r2 = 0.f, rc = 0.f;
#pragma unroll
  for (int k = 0; k < MAX_ITEMS; ++k) {
    const int t = tid + k * BLOCK;
    if (k > 0) {
      ph += pstep;
      ph -= (ph >= m) ? m : 0;
    }
    if (t < T) {
      const float se = pm[ph];
      const float r = D[t] - se;
      if (a.seasonal) a.seasonal[base + t] = se;
      if (a.resid) a.resid[base + t] = r;
      if (r == r) { r2 += r * r; rc += 1.f; }
    }
  }
  if (a.det.C <= 0 && !a.sigma) return;

  // 5. scoring: trend extrapolated from its last defined value over the last season
  const float rss = block_sum(r2, red), rcnt = block_sum(rc, red);
  const float sig = sqrtf(rss / fmaxf(rcnt, 1.f));
  const float lvl = tr_e == tr_e ? tr_e : ybar;
  const float slope = (tr_e == tr_e && tr_p == tr_p) ? (tr_e - tr_p) / (float)m : 0.f;
  if (tid == 0) {
    if (a.fc_level) a.fc_level[n] = lvl;
    if (a.fc_slope) a.fc_slope[n] = slope;
    if (a.sigma) a.sigma[n] = sig;
    if (a.nvalid) a.nvalid[n] = csum;
  }
  const int tlast = T - 1;
  detect_epilogue(a.det, n, sig, csum, [&](int hz) {
    const int p = (tlast + hz) % m;
    return lvl + slope * (float)(tlast + hz - te) + pm[p < 0 ? p + m : p];
  }, red);
}

}  // namespace

extern "C" size_t fm_decompose_lds_bytes(int T, int m) {
  return (size_t)((T + 1) + m + 2 * (BLOCK / FM_WAVE)) * sizeof(float) + (((size_t)(T + 1) * 2 + 3) & ~(size_t)3);
}

extern "C" long long fm_decompose_args_size() { return (long long)sizeof(DecompArgs); }

extern "C" int fm_seasonal_decompose(const DecompArgs* a, hipStream_t st) {
  if (a->N <= 0) return 0;
  if (a->m < 2 || a->T < 2 * a->m || a->T > a->ring_len || a->head < 0 || a->head >= a->ring_len ||
      a->T > BLOCK * MAX_ITEMS)
    return (int)hipErrorInvalidValue;
  const size_t lds = fm_decompose_lds_bytes(a->T, a->m);
  if (lds > 160 * 1024) return (int)hipErrorInvalidValue;
  if (a->bf16)
    hipLaunchKernelGGL(decompose_kernel<bf16_t>, dim3(a->N), dim3(BLOCK), lds, st, *a);
  else
    hipLaunchKernelGGL(decompose_kernel<float>, dim3(a->N), dim3(BLOCK), lds, st, *a);
  return (int)hipGetLastError();
}
