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
__global__ __launch_bounds__(BLOCK, KT <= kItemsWeek ? 8 : 4) void decompose_kernel(const DecompArgs a) {
  const int n = blockIdx.x;
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

}  // namespace

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
  // register-resident items: 20 per thread covers a 7-day window of 60 s points (10,080)
  const int kt = (a->T + BLOCK - 1) / BLOCK;
  const bool small = kt <= kItemsWeek;
#define FM_DEC_LAUNCH(TIN, KT, EX) \
  hipLaunchKernelGGL((decompose_kernel<TIN, KT, EX>), dim3(a->N), dim3(BLOCK), lds, st, *a)
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
  return (int)hipGetLastError();
}
