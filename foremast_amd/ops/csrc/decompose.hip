// K4: classical additive seasonal decomposition (trend / seasonal / resid)
// of every series of a history ring, one workgroup per series.
//
// Semantics: foremast_amd/models/decompose.py (NaN-aware 2 x m centred MA
// trend, centred per-phase means of the detrended series, residual).
//
// Schedule (512 threads, the series read from HBM exactly once, never staged):
//  0. coalesced loads of the ring window (all of a thread's loads in flight at
//     once; sample t = tid + k*512 stays in register k) + block mean of the
//     valid values (the offset that keeps the fp32 prefix sums small — the MA
//     is a difference of two prefix sums);
//  1. exclusive prefix of valid*(y - mean) straight from the registers: per
//     item a DPP wave scan over 64 consecutive samples (row_shr + row_bcast,
//     no LDS traffic), the 64-sample block totals and validity ballots to LDS,
//     one wave scans the block totals, every sample writes its prefix once
//     (consecutive lanes, conflict-free).  Valid counts are not stored per
//     sample: count(i) = valid samples before i's 64-block + popcount of the
//     block's ballot below i, and a gap-free window (the common case) skips
//     even that (count(i) = i);
//  2. trend per sample from the prefix sums (O(1) each), kept in registers;
//     the detrended series overwrites the prefix array;
//  3. per phase p (strided over threads): mean over periods of y - trend;
//  4. one coalesced output pass: seasonal = phase_mean[t mod m], resid (the
//     trend is stored in pass 2).  LDS: 4 (T+1) + 4 m + 16 T/64 bytes
//     (47 KiB at T = 10080, m = 1440), so three workgroups share a CU.
//     (Round 1 staged the series in LDS, scanned per-thread contiguous chunks
//     — a 20-float stride, 8-way bank conflicts — and kept a uint16 count
//     prefix: 66 KiB, two workgroups per CU, 5.8 ms per 100k x 10,080.)
//
// Scoring mode (det.C > 0, the ML_ALGORITHM=seasonal_decompose scorer): the residual RMS
// is reduced in pass 4 and the forecast f(h) = trend_e + slope (T - 1 + h - t_e) +
// seasonal[(T - 1 + h) mod m] (t_e: the last sample with a centred-MA trend, slope over
// the last season of trend) runs through the shared band / verdict epilogue (detect.h);
// with the full outputs null, a series costs one HBM read and no [N, T] writes.
#include "common.h"
#include "args.h"
#include "detect.h"

#include <type_traits>

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
  int* defer;         // scoring fast path: [N + 2] count, series the general kernel finishes, finished
                      // workgroups of that launch (both counts zero between launches); or null
  float* sfc;         // fast path, split epilogue: [N, hmax] seasonal term of horizons 1..hmax, or null
  int hmax;           // (sfc) every horizon is in 1..hmax <= 64
  int _pad;
};

extern __shared__ __attribute__((aligned(16))) char fm_dec_smem[];

namespace {

constexpr int BLOCK = 1024;
constexpr int NW = BLOCK / FM_WAVE;  // waves per workgroup
constexpr int MAX_ITEMS = 16;        // samples per thread held in registers: T <= 16384
constexpr int kItemsWeek = 10;       // T <= 10240

template <typename TIN>
__device__ __forceinline__ float load_y(const DecompArgs& a, const TIN* row, int i) {
  int c = a.head + i;
  if (c >= a.ring_len) c -= a.ring_len;
  return to_f32<TIN>(row[c]);
}

template <int CTRL, int RM>
__device__ __forceinline__ float dppf(float old, float src) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(src), CTRL, RM, 0xf, false));
}

// inclusive wave scan: row scans (row_shr 1/2/4/8, out-of-row sources read as 0), then
// row_bcast 15 / 31 carry the row totals up
__device__ __forceinline__ float wave_inclusive_scan(float v) {
  v += dppf<0x111, 0xf>(0.f, v);
  v += dppf<0x112, 0xf>(0.f, v);
  v += dppf<0x114, 0xf>(0.f, v);
  v += dppf<0x118, 0xf>(0.f, v);
  v += dppf<0x142, 0xa>(0.f, v);
  v += dppf<0x143, 0xc>(0.f, v);
  return v;
}

__device__ __forceinline__ v2f block_sum2(v2f v, float* red) {
  v = wave_sum2(v);
  const int w = wave_id();
  __syncthreads();
  if (lane_id() == 0) { red[2 * w] = v.x; red[2 * w + 1] = v.y; }
  __syncthreads();
  v2f s = {0.f, 0.f};
#pragma unroll
  for (int i = 0; i < NW; ++i) { s.x += red[2 * i]; s.y += red[2 * i + 1]; }
  return s;
}

__device__ __forceinline__ float block_sum(float v, float* red) {
  v2f p = {v, 0.f};
  return block_sum2(p, red).x;
}

// LDS layout (bytes): validity masks [NB] u64 | S [T+1] f32 | phase means [m] f32 |
// red [2 NW] f32 | block sums [NB] f32 | block count offsets [NB] i32,  NB = 64-sample blocks
__host__ __device__ __forceinline__ int dec_blocks(int T) { return ((T + BLOCK - 1) / BLOCK) * NW; }

// EXACT: the launch guarantees ceil(T / BLOCK) == KT, so every item but the last is
// in range at compile time (fewer per-item scalar guards and SGPR pairs live)
template <typename TIN, int KT, bool EXACT>
__device__ __forceinline__ void decompose_series(const DecompArgs& a, const int n) {
  const TIN* row = (const TIN*)a.hist + (long long)n * a.ld;
  const int T = a.T, m = a.m, tid = threadIdx.x, lane = lane_id(), w = wave_id();
  const int NB = dec_blocks(T);
  auto live = [&](int k) { return (EXACT && k < KT - 1) || k * BLOCK < T; };
  unsigned long long* msk = (unsigned long long*)fm_dec_smem;  // bit l of block b: sample 64 b + l valid
  float* S = (float*)(msk + NB);     // [T+1] exclusive prefix of valid*(y - ybar), then the detrended series
  float* pm = S + (T + 1);           // [m]
  float* red = pm + m;               // [2 * NW]
  float* bsum = red + 2 * NW;        // [NB] sum of block b, then its exclusive offset
  int* coff = (int*)(bsum + NB);     // [NB] valid samples before block b

  // 0. coalesced loads (all of a thread's loads in flight at once, clamped index); sample
  //    t = tid + k*BLOCK stays in register yr[k] until the detrended series is formed.
  //    Sample t is lane (t & 63) of wave (t >> 6) & 7 in item t >> 9, so every wave-level
  //    scan below runs over 64 consecutive samples.
  float yr[KT];
#pragma unroll
  for (int k = 0; k < KT; ++k)
    if (live(k)) yr[k] = load_y<TIN>(a, row, min(tid + k * BLOCK, T - 1));
  // scoring mode: touch the epilogue's per-series inputs now (current points, horizons,
  // thresholds) so their cache lines arrive with the samples; the epilogue at the end then
  // hits L2 instead of waiting on a chain of HBM round trips after the last barrier
  float pre = 0.f;
  if (a.det.C > 0) {
    const DetectArgs& d = a.det;
    if (tid < d.C) {
      if (d.cur) pre += d.cur[(long long)n * d.ld_cur + tid];
      pre += (float)d.horizons[d.h_ld * n + tid];
    }
    if (tid == 0) {
      pre += d.threshold[n] + d.min_lower[n] + (float)d.bound[n];
      if (d.threshold_low) pre += d.threshold_low[n];
      if (d.differs) pre += (float)d.differs[n];
    }
  }
  v2f sc = {0.f, 0.f};
#pragma unroll
  for (int k = 0; k < KT; ++k) {
    const int t = tid + k * BLOCK;
    if (t < T && yr[k] == yr[k]) { sc.x += yr[k]; sc.y += 1.f; }
  }
  const v2f tot = block_sum2(sc, red);
  const float csum = tot.y;
  const float ybar = csum > 0.f ? tot.x / csum : 0.f;
  // no gap in this series' window (the common case): in an SGPR, so the gap-free trend pass
  // below is a scalar branch, not both paths under an exec mask
  const bool allvalid = __builtin_amdgcn_readfirstlane((int)(csum == (float)T)) != 0;

  // 1. prefix sums in registers: per item a DPP wave scan over 64 consecutive samples; the
  //    block totals (and validity ballots) go to LDS and one wave scans them
#pragma unroll
  for (int k = 0; k < KT; ++k) {
    if (live(k)) {
      const int t = tid + k * BLOCK;
      const bool ok = t < T && yr[k] == yr[k];
      const float v = ok ? yr[k] - ybar : 0.f;
      const float inc = wave_inclusive_scan(v);
      const unsigned long long b = __ballot(ok);
      if (t < T) S[t] = inc - v;  // exclusive within the 64-sample block
      if (lane == FM_WAVE - 1) bsum[k * NW + w] = inc;
      if (lane == 0) { msk[k * NW + w] = b; coff[k * NW + w] = __popcll(b); }
    }
  }
  __syncthreads();
  if (w == 0) {
    // exclusive scan of the NB block (sum, count) pairs: each lane a run of consecutive blocks
    const int per = (NB + FM_WAVE - 1) / FM_WAVE;
    const int b0 = min(NB, lane * per), b1 = min(NB, b0 + per);
    float ls = 0.f;
    int lc = 0;
    for (int b = b0; b < b1; ++b) { ls += bsum[b]; lc += coff[b]; }
    const float is = wave_inclusive_scan(ls);
    const float ic = wave_inclusive_scan((float)lc);  // exact: counts < 2^24
    float rs = is - ls;
    int rc = (int)(ic - (float)lc);
    for (int b = b0; b < b1; ++b) {
      const float s = bsum[b];
      const int c = coff[b];
      bsum[b] = rs;
      coff[b] = rc;
      rs += s;
      rc += c;
    }
    if (lane == FM_WAVE - 1) S[T] = is;
  }
  __syncthreads();
  // block offsets into the prefix (each thread its own samples: conflict-free read-modify-write)
#pragma unroll
  for (int k = 0; k < KT; ++k) {
    const int t = tid + k * BLOCK;
    if (live(k) && t < T) S[t] += bsum[k * NW + w];
  }
  __syncthreads();

  asm volatile("" ::"v"(pre));  // the prefetch above retires here, long after it landed

  // valid samples before i (0 <= i <= T): block offset + popcount of the lower mask bits
  auto cn = [&](int i) -> float {
    if (allvalid) return (float)i;
    if (i >= T) return csum;
    const int b = i >> 6;
    return (float)(coff[b] + __popcll(msk[b] & ((1ull << (i & 63)) - 1ull)));
  };
  const int h = m / 2;
  const bool even = (m & 1) == 0;
  const float inv_m = 1.f / (float)m;
  // trend at t (NaN at the edges / when < half the window is valid)
  auto trend_at = [&](int t) -> float {
    if (t < h || t + h > T - 1) return fm_nan();
    float num, den;
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
  //    barrier S is free and becomes the detrended series D (each register holds
  //    y - trend from here on; the trend output is stored here, so its 4 bytes per sample leave while the
  //    workgroup still has the phase-mean pass to do)
  const long long base = (long long)n * T;
  // gap-free window: every 2 x m window is complete (weight sum m), so the trend is the
  // prefix difference over m; indices clamped into range and the edges selected to NaN
  // (branch-free per lane)
  auto full_pass = [&](auto EV, auto ST) {
    constexpr bool EVEN = decltype(EV)::value, STORE = decltype(ST)::value;
#pragma unroll
    for (int k = 0; k < KT; ++k) {
      const int t = tid + k * BLOCK;
      if (live(k) && t < T) {
        const int tc = min(max(t, h), T - 1 - h);
        const float num = EVEN ? 0.5f * ((S[tc + h] + S[tc + h + 1]) - (S[tc - h] + S[tc - h + 1]))
                               : S[tc + h + 1] - S[tc - h];
        const float tr = (t < h || t + h > T - 1) ? fm_nan() : ybar + num * inv_m;
        if (STORE) a.trend[base + t] = tr;
        yr[k] -= tr;  // the sample's register now holds the detrended value
      }
    }
  };
  if (allvalid) {
    if (even) {
      if (a.trend) full_pass(std::true_type{}, std::true_type{});
      else full_pass(std::true_type{}, std::false_type{});
    } else {
      if (a.trend) full_pass(std::false_type{}, std::true_type{});
      else full_pass(std::false_type{}, std::false_type{});
    }
  } else {
#pragma unroll
    for (int k = 0; k < KT; ++k) {
      const int t = tid + k * BLOCK;
      if (live(k) && t < T) {
        const float tr = trend_at(t);
        if (a.trend) a.trend[base + t] = tr;
        yr[k] -= tr;
      }
    }
  }
  // scoring mode: the last defined trend and the one a season earlier (every thread, from
  // the prefix sums, before they are overwritten)
  const int te = T - 1 - h;
  const float tr_e = trend_at(te), tr_p = te - m >= 0 ? trend_at(te - m) : fm_nan();
  __syncthreads();
  float* D = S;
#pragma unroll
  for (int k = 0; k < KT; ++k) {
    const int t = tid + k * BLOCK;
    if (live(k) && t < T) D[t] = yr[k];
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
  float r2 = 0.f, rc = 0.f;
  auto out_pass = [&](auto ST) {
    constexpr bool STORE = decltype(ST)::value;  // full outputs (both or neither: see below)
    int ph = tid % m;
#pragma unroll
    for (int k = 0; k < KT; ++k) {
      const int t = tid + k * BLOCK;
      if (k > 0) {
        ph += pstep;
        ph -= (ph >= m) ? m : 0;
      }
      if (live(k) && t < T) {
        const float se = pm[ph];
        const float r = D[t] - se;
        if (STORE) {
          if (a.seasonal) a.seasonal[base + t] = se;
          if (a.resid) a.resid[base + t] = r;
        }
        if (r == r) { r2 += r * r; rc += 1.f; }
      }
    }
  };
  if (a.seasonal || a.resid) out_pass(std::true_type{});
  else out_pass(std::false_type{});
  if (a.det.C <= 0 && !a.sigma) return;

  // 5. scoring: trend extrapolated from its last defined value over the last season
  const v2f rr = block_sum2(v2f{r2, rc}, red);
  const float rss = rr.x, rcnt = rr.y;
  // residual RMS -> prediction spread of the phase-mean model (models/decompose.py
  // prediction_factor): sqrt((K+1)/(K-1)), K = seasons with a centred trend
  const float Ks = fmaxf((float)(T - 2 * h) / (float)m, 1.5f);
  const float sig = sqrtf(rss / fmaxf(rcnt, 1.f)) * sqrtf((Ks + 1.f) / (Ks - 1.f));
  const float lvl = tr_e == tr_e ? tr_e : ybar;
  const float slope = (tr_e == tr_e && tr_p == tr_p) ? (tr_e - tr_p) / (float)m : 0.f;
  if (tid == 0) {
    if (a.fc_level) a.fc_level[n] = lvl;
    if (a.fc_slope) a.fc_slope[n] = slope;
    if (a.sigma) a.sigma[n] = sig;
    if (a.nvalid) a.nvalid[n] = csum;
  }
  // band / verdict: one wave (lanes stride the columns, wave reductions) — the block
  // version's dozen workgroup barriers cost more than the 50-odd columns themselves
  if (w != 0) return;
  const int tlast = T - 1;
  detect_epilogue_wave(a.det, n, sig, csum, [&](int hz) {
    const int p = (tlast + hz) % m;
    return lvl + slope * (float)(tlast + hz - te) + pm[p < 0 ? p + m : p];
  });
}

template <typename TIN, int KT, bool EXACT>
__global__ __launch_bounds__(BLOCK, KT <= kItemsWeek ? 8 : 4) void decompose_kernel(const DecompArgs a) {
  decompose_series<TIN, KT, EXACT>(a, blockIdx.x);
}

// out of line: inlined into the loop below, LLVM hoists every per-item invariant out of it
// and spills hundreds of registers
template <typename TIN, int KT, bool EXACT>
__device__ __attribute__((noinline)) void decompose_series_call(const DecompArgs& a, int n) {
  decompose_series<TIN, KT, EXACT>(a, n);
}

// the series the scoring fast path deferred (a gap or a non-finite value in the window):
// a grid-stride loop over the device-side list (the count is only known on the device).
// Every wave runs every iteration (the early returns above are per call), and nothing in a
// call writes LDS before its first workgroup barrier, so calls follow each other safely.
template <typename TIN, int KT, bool EXACT>
__global__ __launch_bounds__(BLOCK, 4) void decompose_deferred_kernel(const DecompArgs a) {
  const int cnt = min(a.defer[0], a.N);
  for (int q = blockIdx.x; q < cnt; q += gridDim.x) {
    decompose_series_call<TIN, KT, EXACT>(a, a.defer[1 + q]);
    __syncthreads();
  }
  // the last workgroup out resets the count for the next launch (every workgroup has read
  // it by then): no memset launch per call.  defer[N + 1] counts the finished workgroups.
  if (threadIdx.x == 0) {
    __threadfence();
    if (atomicAdd(&a.defer[a.N + 1], 1) == (int)gridDim.x - 1) {
      atomicExch(&a.defer[0], 0);
      atomicExch(&a.defer[a.N + 1], 0);
    }
  }
}

// ---- scoring fast path: one streaming pass ------------------------------------------
// ML_ALGORITHM=seasonal_decompose scores with the forecast, the residual RMS and the band;
// none of the [N, T] outputs.  For a gap-free window with an even period (m % 16 == 0) the
// whole decomposition collapses to:
//  * P = inclusive prefix of y - y0 (8 consecutive samples per lane from one 16-byte load,
//    in-lane prefix, one DPP wave scan per 8 samples, block offsets), written once to LDS;
//  * D_t = y_t - trend_t = (P[t] - P[t-1]) - (d[t-1] + d[t]) / 2m with d[j] = P[j+h] - P[j-h]
//    (the 2 x m centred window as two prefix differences), 8 samples of a lane at once:
//    D_i = g_i - e_{i-1} with g = P - d/2m, e = P + d/2m (packed FP32; e_{-1} is the
//    neighbour lane's e_7, one DPP move — no strided LDS reads);
//  * per phase p (consecutive lanes, conflict-free): the mean pm_p of D over the periods with
//    a centred trend and W_p = sum (D - pm_p)^2.  With the seasonal s_p = pm_p - pmean the
//    residual sum of squares is sum_p W_p + pmean^2 * count (the cross term vanishes), so no
//    residual pass and no cancellation.  The 7-day / daily geometry (T = 7 m, m = 1440) is
//    compiled with its period: every phase has exactly 6 centred periods at immediate offsets.
// Persistent workgroups (3 per CU, the LDS bound) walk the series with a stride of the grid
// and issue the next series' loads before working on the current one, so HBM latency hides
// under the LDS passes.  With a host-known horizon bound the band / verdict runs in its own
// kernel (decompose_detect_kernel) from the seasonal terms left here, off this loop's
// critical path.  A window with a NaN/Inf has a non-finite prefix total: its series is
// appended to `defer` and the general kernel above finishes it (identical semantics, gaps
// included).  The ring head moves one column per tick: t' = t + (head mod 8) keeps every
// 8-group of samples one aligned vector load (the columns outside the window are zeros).
constexpr int SB = 448;             // threads per workgroup (7 waves: 3 x 3,584 samples cover 7 days)
constexpr int SNW = SB / FM_WAVE;
constexpr int SE = 8;               // consecutive samples per lane and item
constexpr int S_MAX_ITEMS = 5;      // T + 14 <= 17,920
constexpr int S_WG_PER_CU = 3;      // 49 KiB of LDS per workgroup at T = 10,080

struct v8f { v4f lo, hi; };

template <typename TIN> struct Raw8;  // the raw bits of 8 consecutive samples
template <> struct Raw8<bf16_t> {
  uint4 u;
  __device__ __forceinline__ void load(const bf16_t* p) { u = *(const uint4*)p; }
  __device__ __forceinline__ void zero() { u = make_uint4(0u, 0u, 0u, 0u); }
  __device__ __forceinline__ v8f get() const {
    v8f r;
    r.lo = v4f{__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
               __uint_as_float(u.y & 0xffff0000u)};
    r.hi = v4f{__uint_as_float(u.z << 16), __uint_as_float(u.z & 0xffff0000u), __uint_as_float(u.w << 16),
               __uint_as_float(u.w & 0xffff0000u)};
    return r;
  }
};
template <> struct Raw8<float> {
  v4f a, b;
  __device__ __forceinline__ void load(const float* p) { a = *(const v4f*)p; b = *(const v4f*)(p + 4); }
  __device__ __forceinline__ void zero() { a = b = v4f{0.f, 0.f, 0.f, 0.f}; }
  __device__ __forceinline__ v8f get() const { return v8f{a, b}; }
};

// items per thread of the instantiated kernel (1..5) for a window of T samples
__host__ __device__ __forceinline__ int score_items(int T) { return (T + 14 + SB * SE - 1) / (SB * SE); }

// the kernel arguments in the constant address space: reads are scalar loads (a generic
// pointer would turn them into flat loads whose waits also drain the prefetched samples)
typedef const __attribute__((address_space(4))) DecompArgs* KArgs;

// the detection arguments as a register value (word-wise scalar loads from the kernarg segment)
__device__ __forceinline__ DetectArgs kdet(KArgs a) {
  static_assert(sizeof(DetectArgs) % 4 == 0, "word copy");
  DetectArgs d;
  const __attribute__((address_space(4))) int* src = (const __attribute__((address_space(4))) int*)&a->det;
  int* dst = (int*)&d;
#pragma unroll
  for (int i = 0; i < (int)(sizeof(DetectArgs) / 4); ++i) dst[i] = src[i];
  return d;
}

// y0: the raw first sample, converted only when the series is worked on (converting it here
// would wait for the load, and with it for every prefetched sample)
template <typename TIN, int KT>
__device__ __forceinline__ void score_issue(KArgs a, int n, Raw8<TIN>* raw, TIN& y0) {
  const TIN* row = (const TIN*)a->hist + (long long)n * a->ld;
  const int head = a->head, phi = head & 7, TP = a->T + phi, col0 = head - phi, R = a->ring_len;
  y0 = row[head];
#pragma unroll
  for (int k = 0; k < KT; ++k) {
    const int tg = (threadIdx.x + k * SB) * SE;
    raw[k].zero();
    if (tg < TP) {
      int c = col0 + tg;
      c -= (c >= R) ? R : 0;
      raw[k].load(row + c);
    }
  }
}

__device__ __forceinline__ float wave_shr1(float old, float v) {  // lane l <- lane l-1 (lane 0: old)
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(v), 0x138, 0xf, 0xf, false));
}

// M > 0: the compiled geometry T = 7 M (host-checked); M = 0: any period with m % 16 == 0
// (the general-period variants need more registers: two workgroups per CU)
template <typename TIN, int KT, int M>
__global__ __launch_bounds__(SB, M > 0 ? 6 : 4) void decompose_score_kernel(const DecompArgs a0) {
  const KArgs a0p = (KArgs)__builtin_amdgcn_kernarg_segment_ptr();
  const int T = a0.T, m = M > 0 ? M : a0.m, h = m >> 1;
  const int tid = threadIdx.x, lane = lane_id(), w = wave_id();
  const int phi = a0.head & 7, TP = T + phi;
  float* P = (float*)fm_dec_smem + 4;  // [-4, KT SB SE): inclusive prefix of y - y0, then D
  float* pmv = P + KT * SB * SE;       // [m] phase means
  float* red = pmv + m;                // [4 SNW] reductions, [4 SNW] prefix total
  float* bsum = red + 8 * SNW;         // [KT SNW] wave totals, then their exclusive offsets
  const float cm = 0.5f / (float)m;
  const int te = T - 1 - h;
  const int lo = h, hi = (te + phi) & ~7;
  if (tid < 4) P[tid - 4] = 0.f;

  Raw8<TIN> nxt[KT];
  TIN y0n = 0;
  int n = blockIdx.x;
  if (n < a0.N) score_issue<TIN, KT>(a0p, n, nxt, y0n);
  for (; n < a0.N; n += gridDim.x) {
    // the arguments are re-read from the kernarg segment where they are used (scalar loads):
    // hoisted out of the loop they hold ~100 SGPRs live across it and spill
    KArgs a = a0p;
    asm volatile("" : "+s"(a));
    // lane-derived addresses are recomputed per series (hoisted, ~20 VGPRs live across the
    // loop spill, and a spill reload's wait drains the prefetched samples)
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    Raw8<TIN> raw[KT];
#pragma unroll
    for (int k = 0; k < KT; ++k) raw[k] = nxt[k];
    const float y0 = to_f32<TIN>(y0n);
    if (n + (int)gridDim.x < a->N) score_issue<TIN, KT>(a, n + gridDim.x, nxt, y0n);  // block-uniform

    // 1. prefix: in-lane inclusive over 8 samples, DPP wave scan of the lane totals; the
    //    samples (y - y0, masked) stay in registers through the block scan and the prefix is
    //    written once, offsets included (recomputing the 7 in-lane adds is cheaper than an
    //    LDS read-modify-write pass)
    v8f v[KT];
    float ex[KT];
#pragma unroll
    for (int k = 0; k < KT; ++k) {
      const int tg = (tid + k * SB) * SE;
      v8f q = raw[k].get();
      q.lo -= y0;
      q.hi -= y0;
      if (tg < phi || tg + SE > TP) {  // the window's edge groups: columns outside it are 0
        float e[8] = {q.lo.x, q.lo.y, q.lo.z, q.lo.w, q.hi.x, q.hi.y, q.hi.z, q.hi.w};
#pragma unroll
        for (int i = 0; i < 8; ++i) e[i] = (tg + i >= phi && tg + i < TP) ? e[i] : 0.f;
        q.lo = v4f{e[0], e[1], e[2], e[3]};
        q.hi = v4f{e[4], e[5], e[6], e[7]};
      }
      v[k] = q;
      const float tot = ((q.lo.x + q.lo.y) + (q.lo.z + q.lo.w)) + ((q.hi.x + q.hi.y) + (q.hi.z + q.hi.w));
      const float inc = wave_inclusive_scan(tot);
      ex[k] = inc - tot;
      if (lane == FM_WAVE - 1) bsum[k * SNW + w] = inc;
    }
    __syncthreads();
    if (w == 0) {
      const float b = lane < KT * SNW ? bsum[lane] : 0.f;
      const float inc = wave_inclusive_scan(b);
      if (lane < KT * SNW) bsum[lane] = inc - b;
      if (lane == KT * SNW - 1) red[4 * SNW] = inc;
    }
    __syncthreads();
    const float total = red[4 * SNW];
    if (!__builtin_isfinite(total)) {  // block-uniform: a gap or a non-finite sample
      if (tid == 0) {
        const int q = atomicAdd(a->defer, 1);
        if (q < a->N) a->defer[1 + q] = n;
        if (a->sfc) a->sfc[(long long)n * a->hmax] = fm_nan();  // the detect kernel skips it
      }
      continue;
    }
#pragma unroll
    for (int k = 0; k < KT; ++k) {
      const int tg = (tid + k * SB) * SE;
      v8f q = v[k];
      q.lo.x += ex[k] + bsum[k * SNW + w];
      q.lo.y += q.lo.x;
      q.lo.z += q.lo.y;
      q.lo.w += q.lo.z;
      q.hi.x += q.lo.w;
      q.hi.y += q.hi.x;
      q.hi.z += q.hi.y;
      q.hi.w += q.hi.z;
      *(v4f*)(P + tg) = q.lo;
      *(v4f*)(P + tg + 4) = q.hi;
    }
    __syncthreads();

    // 2. detrended samples, in place of the samples: D_i = v_i - (d_i + d_{i-1}) / 2m with
    //    d_j = P[j+h] - P[j-h] (the groups without a centred trend read a clamped, in-range
    //    position and are never used); d_{-1} comes from the previous lane (its group is the
    //    adjacent one) except in lane 0 and at the lower clamp, which read it
#pragma unroll
    for (int k = 0; k < KT; ++k) {
      const int tg = (tid + k * SB) * SE;
      const int tc = min(max(tg, lo), hi);
      v4f d0 = *(const v4f*)(P + tc + h), d1 = *(const v4f*)(P + tc + h + 4);
      d0 -= *(const v4f*)(P + tc - h);
      d1 -= *(const v4f*)(P + tc - h + 4);
      const bool own = lane == 0 || tg <= lo;
      float dm = 0.f;
      if (own) dm = P[tc + h - 1] - P[tc - h - 1];
      const float dsh = wave_shr1(dm, d1.w);
      dm = own ? dm : dsh;
      v[k].lo -= cm * (d0 + v4f{dm, d0.x, d0.y, d0.z});
      v[k].hi -= cm * (d1 + v4f{d0.w, d1.x, d1.y, d1.z});
      // the item is finished before the next one's LDS reads issue (all in flight: spills)
      asm volatile("" : "+v"(v[k].lo), "+v"(v[k].hi)::"memory");
    }
    // the forecast's trend anchors: the last centred trend and the one a season earlier
    float tr_e = 0.f, tr_p = 0.f;
    if (w == 0) {
      auto trend_at = [&](int t) {
        const int u = t + phi;
        return y0 + cm * ((P[u + h - 1] + P[u + h]) - (P[u - h - 1] + P[u - h]));
      };
      tr_e = trend_at(te);
      tr_p = trend_at(te - m);
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < KT; ++k) {
      const int tg = (tid + k * SB) * SE;
      if (tg < TP) {
        *(v4f*)(P + tg) = v[k].lo;
        *(v4f*)(P + tg + 4) = v[k].hi;
      }
    }
    __syncthreads();

    // 3. per phase: mean over the periods with a centred trend, squared deviations from it
    float spm = 0.f, sw = 0.f, sc = 0.f;
    if constexpr (M > 0) {  // T = 7 M: periods 1..6 for p < h, 0..5 otherwise — 6 at immediate offsets
      constexpr float inv6 = 1.f / 6.f;
      constexpr int NP = M > 0 ? (M + SB - 1) / SB : 1;
#pragma unroll
      for (int j = 0; j < NP; ++j) {
        const int p = tid + j * SB;
        if (j * SB + SB <= M || p < M) {
          const float* d = P + p + phi + (p < h ? M : 0);
          float v6[6];
#pragma unroll
          for (int k = 0; k < 6; ++k) v6[k] = d[k * M];
          const float pm = (((v6[0] + v6[1]) + (v6[2] + v6[3])) + (v6[4] + v6[5])) * inv6;
          float ww = 0.f;
#pragma unroll
          for (int k = 0; k < 6; ++k) {
            const float e = v6[k] - pm;
            ww += e * e;
          }
          pmv[p] = pm;
          spm += pm;
          sw += ww;
        }
      }
      sc = (float)(6 * (M / SB) + (tid < M % SB ? 6 : 0));
    } else {
      for (int p = tid; p < m; p += SB) {
        const int k0 = p < h ? 1 : 0, k1 = (te - p) / m;
        const float* d = P + p + phi;
        float s = 0.f;
        for (int k = k0; k <= k1; ++k) s += d[k * m];
        const float cnt = (float)(k1 - k0 + 1);
        const float pm = s * __builtin_amdgcn_rcpf(cnt);
        float ww = 0.f;
        for (int k = k0; k <= k1; ++k) {
          const float e = d[k * m] - pm;
          ww += e * e;
        }
        pmv[p] = pm;
        spm += pm;
        sw += ww;
        sc += cnt;
      }
    }
    spm = wave_allsum(spm);
    sw = wave_allsum(sw);
    sc = wave_allsum(sc);
    if (lane == 0) { red[w] = spm; red[SNW + w] = sw; red[2 * SNW + w] = sc; }
    __syncthreads();
    float tpm = 0.f, tw = 0.f, tcnt = 0.f;
#pragma unroll
    for (int i = 0; i < SNW; ++i) { tpm += red[i]; tw += red[SNW + i]; tcnt += red[2 * SNW + i]; }
    const float pmean = tpm / (float)m;
    const float rss = tw + pmean * pmean * tcnt;
    if (a->phase_means)
      for (int p = tid; p < m; p += SB) a->phase_means[(long long)n * m + p] = pmv[p] - pmean;

    // 4. forecast parameters, spread, band / verdict (wave 0; the other waves go on to the
    //    next series, whose first LDS writes cannot touch pmv before wave 0 has joined them).
    //    Split epilogue (sfc): only the seasonal terms of horizons 1..hmax leave here.
    if (w == 0) {
      // (float) T and the lane's seasonal-term address are derived here, per series: hoisted
      // out of the loop they were spilled, and the reload's vmcnt(0) drained the next
      // series' prefetched samples (the trap the argument / tid laundering above avoids)
      int Tn = T;
      asm volatile("" : "+s"(Tn));
      const float Tf = (float)Tn;
      const int ln = tid & (FM_WAVE - 1);
      const float Ks = fmaxf((float)(T - 2 * h) / (float)m, 1.5f);
      const float sig = sqrtf(rss / fmaxf(tcnt, 1.f)) * sqrtf((Ks + 1.f) / (Ks - 1.f));
      const float slope = (tr_e - tr_p) / (float)m;
      if (ln == 0) {
        if (a->fc_level) a->fc_level[n] = tr_e;
        if (a->fc_slope) a->fc_slope[n] = slope;
        if (a->sigma) a->sigma[n] = sig;
        if (a->nvalid) a->nvalid[n] = Tf;
      }
      const int tlast = Tn - 1;
      if (a->sfc) {
        if (ln < a->hmax) a->sfc[(long long)n * a->hmax + ln] = pmv[(tlast + 1 + ln) % m] - pmean;
        continue;
      }
      const DetectArgs det = kdet(a);
      detect_epilogue_wave(det, n, sig, Tf, [&](int hz) {
        int p = (tlast + hz) % m;
        p += p < 0 ? m : 0;
        return tr_e + slope * (float)(tlast + hz - te) + (pmv[p] - pmean);
      });
    }
  }
}

// split epilogue of the fast path: one 16-lane row per series, the band / verdict from the
// forecast parameters and the seasonal terms the score kernel left (deferred series: NaN
// marker, the general kernel has done their epilogue)
__global__ __launch_bounds__(256) void decompose_detect_kernel(const DecompArgs a) {
  const int n = blockIdx.x * (blockDim.x / 16) + (threadIdx.x >> 4);
  if (n >= a.N) return;  // row-uniform
  const float* sf = a.sfc + (long long)n * a.hmax;
  const float s0 = sf[0];
  if (s0 != s0) return;
  const float lvl = a.fc_level[n], slope = a.fc_slope[n], sig = a.sigma[n], nv = a.nvalid[n];
  const int h = a.m >> 1, hm = a.hmax;
  detect_epilogue_row(a.det, n, sig, nv, [&](int hz) {
    const int i = min(max(hz, 1), hm) - 1;  // the host guarantees 1 <= hz <= hmax
    return lvl + slope * (float)(h + hz) + sf[i];
  });
}

}  // namespace

extern "C" size_t fm_decompose_score_lds_bytes(int T, int m) {
  return ((size_t)4 + (size_t)score_items(T) * SB * SE + m + 8 * SNW + (size_t)score_items(T) * SNW) * sizeof(float);
}

extern "C" size_t fm_decompose_lds_bytes(int T, int m) {
  const size_t nb = (size_t)dec_blocks(T);
  return nb * 8 + ((size_t)(T + 1) + m + 2 * NW + nb) * sizeof(float) + nb * sizeof(int);
}

extern "C" long long fm_decompose_args_size() { return (long long)sizeof(DecompArgs); }

extern "C" int fm_seasonal_decompose(const DecompArgs* a, hipStream_t st) {
  if (a->N <= 0) return 0;
  if (a->m < 2 || a->T < 2 * a->m || a->T > a->ring_len || a->head < 0 || a->head >= a->ring_len ||
      a->T > BLOCK * MAX_ITEMS)
    return (int)hipErrorInvalidValue;
  const size_t lds = fm_decompose_lds_bytes(a->T, a->m);
  if (lds > 160 * 1024) return (int)hipErrorInvalidValue;
  const int ks = score_items(a->T);
  const bool fast = a->defer && !a->trend && !a->seasonal && !a->resid && a->m % 16 == 0 && a->T >= 2 * a->m + 1 &&
                    a->ring_len % 8 == 0 && a->ld % 8 == 0 && (((unsigned long long)a->hist) & 15ull) == 0 &&
                    ks <= S_MAX_ITEMS && fm_decompose_score_lds_bytes(a->T, a->m) <= 160 * 1024 &&
                    (!a->sfc || (a->hmax >= 1 && a->hmax <= FM_WAVE));
  if (fast) {
    hipError_t e;
    const size_t slds = fm_decompose_score_lds_bytes(a->T, a->m);
    static int cus = 0;
    if (!cus) {
      int dev = 0;
      if (hipGetDevice(&dev) != hipSuccess ||
          hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        cus = 256;
    }
    const bool day7 = a->m == 1440 && a->T == 7 * 1440;
    const int wgs = cus * (day7 ? S_WG_PER_CU : 2);
    const int sgrid = a->N < wgs ? a->N : wgs;
#define FM_DEC_SCORE(TIN, KT, M) \
    hipLaunchKernelGGL((decompose_score_kernel<TIN, KT, M>), dim3(sgrid), dim3(SB), slds, st, *a)
#define FM_DEC_SCORE_T(TIN)                                                                       \
    if (day7) FM_DEC_SCORE(TIN, 3, 1440);                                                         \
    else switch (ks) { case 1: FM_DEC_SCORE(TIN, 1, 0); break; case 2: FM_DEC_SCORE(TIN, 2, 0); break; \
                       case 3: FM_DEC_SCORE(TIN, 3, 0); break; case 4: FM_DEC_SCORE(TIN, 4, 0); break; \
                       default: FM_DEC_SCORE(TIN, 5, 0); break; }
    if (a->bf16) { FM_DEC_SCORE_T(bf16_t) } else { FM_DEC_SCORE_T(float) }
#undef FM_DEC_SCORE_T
#undef FM_DEC_SCORE
    e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
  }
  // register-resident items: 20 per thread covers a 7-day window of 60 s points (10,080)
  const int kt = (a->T + BLOCK - 1) / BLOCK;
  const bool small = kt <= kItemsWeek;
  // fast path: the general kernel only finishes the deferred series (grid-stride over the list)
  const int grid = fast ? (a->N < 256 ? a->N : 256) : a->N;
#define FM_DEC_LAUNCH(TIN, KT, EX)                                                                          \
  do {                                                                                                      \
    if (fast) hipLaunchKernelGGL((decompose_deferred_kernel<TIN, KT, EX>), dim3(grid), dim3(BLOCK), lds, st, *a); \
    else hipLaunchKernelGGL((decompose_kernel<TIN, KT, EX>), dim3(grid), dim3(BLOCK), lds, st, *a);         \
  } while (0)
  if (a->bf16) {
    if (kt == kItemsWeek) FM_DEC_LAUNCH(bf16_t, kItemsWeek, true);
    else if (small) FM_DEC_LAUNCH(bf16_t, kItemsWeek, false);
    else FM_DEC_LAUNCH(bf16_t, MAX_ITEMS, false);
  } else {
    if (kt == kItemsWeek) FM_DEC_LAUNCH(float, kItemsWeek, true);
    else if (small) FM_DEC_LAUNCH(float, kItemsWeek, false);
    else FM_DEC_LAUNCH(float, MAX_ITEMS, false);
  }
#undef FM_DEC_LAUNCH
  if (fast && a->sfc && a->det.C > 0) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(decompose_detect_kernel, dim3((a->N + 15) / 16), dim3(256), 0, st, *a);
  }
  return (int)hipGetLastError();
}
