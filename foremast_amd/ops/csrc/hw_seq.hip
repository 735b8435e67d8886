// K3 at short daily seasons: sequential Holt-Winters grid fit with the seasonal state in
// registers, one (series, grid point pair) per thread.
//
// Which steps land here: the create request's `step` sets the daily season m = 86400 / step
// (/root/reference/foremast-service/README.md:26-80; the historical query's 1200 s step
// sketched at /root/reference/foremast-barrelman/pkg/client/metrics/metricsquery.go:74).
// m = 72 (1200 s), 24 (3600 s), 48 (1800 s), 96 (900 s) and 144 (600 s) are too short for the
// time-parallel schedule of hw_scan.hip to pay: a season of 72 is 32 lanes x 2.25 steps, so
// the per-season scan and its carry passes would cost more than the walk itself.  At these
// seasons the whole seasonal state of a grid point fits in VGPRs (m floats), so the fit is
// what es_seq.hip does for ES / DES, with the season added: every thread walks its series
// from LDS for two grid points at once (packed FP32; one grid point per thread at m = 144),
// s[t mod m] indexed at compile time inside a fully unrolled season.
//
// Same semantics as models/smoothing.py (MODE_HW): front padding with NaN to a multiple of m;
// season 0 initialises l0 = nanmean(season 0), b0 = (nanmean(season 1) - l0) / m,
// s[p] = y[p] - l0 (0 where missing); the fit walks seasons 1 .. Tp/m - 1; a missing point
// carries the forecast (e = 0: no SSE term, no seasonal update); argmin SSE over the grid
// (lowest index on ties); sigma = sqrt(SSE / n_valid).  State in (forecast, trend)
// coordinates: e = (y - s) - f;  f' = (f + b) + c1 e;  b' = b + c2 e;  s' = s + g e, with
// c1 = alpha (1 + beta), c2 = alpha beta, g = gamma (1 - alpha); level = f - b at the end.
//
// Per step and grid-point pair: 7 packed FP32 ops (6 fmas and f + b), a dependency chain of
// two (e, f), gaps included: the staging (one coalesced pass of each workgroup's rows) writes
// two fp32 LDS images, y with a missing point as 0 and a keep factor k (row stride Tp + 4:
// 16-byte ds_reads of four steps), and e = k (y - s - f) costs the same two fmas as
// (y - s) - f (seq_step).  One code path: a branch between a plain and a masked season walk
// kept two copies of the 2 m season registers live (234 VGPRs at m = 48, spills from
// m = 72).  The band / verdict epilogue is fm_hw_detect_params (the fit writes the first
// HALF_HB seasonal phases and the valid count), as for every deferred HW fit.  m = 288 (the
// 300 s step) is instantiated as an opt-in (see seq_gpt).  PMC at m = 72: the season walk is
// ~80 % of the kernel's VALU, which issues in ~83 % of the slots
// (profiles/hw_r6/seq/pmc/).
#include "common.h"
#include "args.h"

#include <cstdlib>

extern __shared__ __attribute__((aligned(16))) char fm_hws_smem[];

extern "C" int fm_hw_detect_params(const SmoothArgs* a, hipStream_t st);

namespace {

constexpr int SEQ_HB = 16;  // seasonal phases written to season_hb (kernels.py HALF_HB)
constexpr int SEQ_LD = 8;   // staging loads in flight per thread
constexpr int SEQ_BUF_DW3 = 0x00020000;  // buffer resource word 3 (raw access) on gfx950

template <int GPT> struct SeqVec;
template <> struct SeqVec<1> { using type = float; };
template <> struct SeqVec<2> { using type = v2f; };

template <typename V> __device__ __forceinline__ V splat_(float a);
template <> __device__ __forceinline__ float splat_<float>(float a) { return a; }
template <> __device__ __forceinline__ v2f splat_<v2f>(float a) { return splat2(a); }

__device__ __forceinline__ float comp_(float v, int) { return v; }
__device__ __forceinline__ float comp_(v2f v, int k) { return k ? v.y : v.x; }

// one step.  yc = y with a missing point as 0, k = 1 observed / 0 missing:
// e = k (y - s - f) = fma(-k, f, fma(-k, s, yc)) is the plain (y - s) - f when k = 1 (an fma
// with -1 rounds like the subtraction) and 0 when k = 0 (a missing point carries the
// forecast: no SSE term, no seasonal update) -- one code path, no per-step mask ops
template <typename V>
__device__ __forceinline__ void seq_step(float yc, float k, V& s, V& f, V& b, V& sse, V c1, V c2, V g) {
  const V nk = splat_<V>(-k);
  const V e = nk * f + (nk * s + splat_<V>(yc));
  const V t = f + b;
  f = t + c1 * e;
  b = b + c2 * e;
  s = s + g * e;
  sse = sse + e * e;
}

// one season from LDS (16-byte reads of four values and four keep factors); p is a
// compile-time index into s
template <int M, typename V>
__device__ __forceinline__ void seq_season(const float* yr, const float* kr, V (&s)[M], V& f, V& b, V& sse, V c1,
                                           V c2, V g) {
#pragma unroll
  for (int p = 0; p < M; p += 4) {
    const v4f y4 = *(const v4f*)(yr + p);
    const v4f k4 = *(const v4f*)(kr + p);
    seq_step(y4.x, k4.x, s[p + 0], f, b, sse, c1, c2, g);
    seq_step(y4.y, k4.y, s[p + 1], f, b, sse, c1, c2, g);
    seq_step(y4.z, k4.z, s[p + 2], f, b, sse, c1, c2, g);
    seq_step(y4.w, k4.w, s[p + 3], f, b, sse, c1, c2, g);
  }
}

// raw bits of one element (bf16: zero-extended), converted after the loads are issued
template <typename TIN> __device__ __forceinline__ unsigned ld_bits(const TIN* p) {
  if constexpr (sizeof(TIN) == 2) return (unsigned)*(const unsigned short*)p;
  else return __float_as_uint(*(const float*)p);
}
template <typename TIN> __device__ __forceinline__ float bits_f32_(unsigned u) {
  return __uint_as_float(sizeof(TIN) == 2 ? u << 16 : u);
}

// A workgroup of 256 threads owns SW = 256 / TPC series; thread gp of a series fits grid
// points GPT gp .. GPT gp + GPT - 1 (clamped to G - 1).  Rows past N stage missing points
// and exit before the walk (a series' TPC threads are whole lane groups, so the shuffles of
// the remaining series never read an exited lane).
template <int M, int GPT, int TPC, typename TIN>
__global__ __launch_bounds__(256, (M > 144 || (M > 96 && GPT == 2)) ? 1 : 2) void hw_seq_kernel(const SmoothArgs a) {
  using V = typename SeqVec<GPT>::type;
  constexpr int SW = 256 / TPC;
  static_assert(M % 4 == 0, "16-byte LDS reads of four steps");
  const int tid = threadIdx.x;
  const int sr = tid / TPC, gp = tid - sr * TPC;
  const int n0 = blockIdx.x * SW, n = n0 + sr;
  const int Tp = a.Tp, pad = a.pad, R = a.ring_len, nseg = Tp / M;
  const int LDY = Tp + 4;
  float* ys = (float*)fm_hws_smem;     // [SW][LDY] padded-time image, a missing point as 0
  float* ks = ys + SW * LDY;            // [SW][LDY] keep factors (1 observed, 0 missing)
  int* nanc = (int*)(ks + SW * LDY);    // [SW] missing points past season 0
  const int head = a.head_dev ? *a.head_dev : a.head;

  if (tid < SW) nanc[tid] = 0;
  __syncthreads();
  // staging: wave w stages rows w, w + 4, ..; lane l columns l, l + 64, ..  (a row's base
  // is wave-uniform, so an element costs a 32-bit offset, no division by Tp).  SEQ_LD loads
  // per lane are in flight before any is converted and stored
  const TIN* base = (const TIN*)a.hist;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6), ln = tid & 63;  // wave-uniform row
  for (int r = wv; r < SW; r += 256 / 64) {
    const int nn = n0 + r;
    const bool rowok = nn < a.N;
    // the row as a raw buffer (wave-uniform descriptor): an element costs a 32-bit offset
    const __amdgpu_buffer_rsrc_t rowb = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(base + (long long)(rowok ? nn : 0) * a.ld), (short)0, (int)(R * (int)sizeof(TIN)), SEQ_BUF_DW3);
    for (int q0 = 0; q0 < Tp; q0 += 64 * SEQ_LD) {
      unsigned u[SEQ_LD];
#pragma unroll
      for (int j = 0; j < SEQ_LD; ++j) {
        const int tau = q0 + 64 * j + ln, t = tau - pad;
        const bool in = rowok && tau < Tp && t >= 0;
        int c = head + t;
        c -= c >= R ? R : 0;
        // unconditional loads (an element outside reads the row's first and is replaced),
        // held by the asm below: a load under a branch is waited for at the branch's join
        const unsigned off = (unsigned)(in ? c : 0) * (unsigned)sizeof(TIN);
        if constexpr (sizeof(TIN) == 2) u[j] = (unsigned)__builtin_amdgcn_raw_buffer_load_b16(rowb, off, 0u, 0);
        else u[j] = __builtin_amdgcn_raw_buffer_load_b32(rowb, off, 0u, 0);
      }
#pragma unroll
      for (int j = 0; j < SEQ_LD; ++j) asm volatile("" : "+v"(u[j]));
#pragma unroll
      for (int j = 0; j < SEQ_LD; ++j) {
        const int tau = q0 + 64 * j + ln, t = tau - pad;
        if (tau < Tp) {
          const float x = (rowok && t >= 0) ? bits_f32_<TIN>(u[j]) : fm_nan();
          const bool ok = x == x;
          ys[r * LDY + tau] = ok ? x : 0.f;
          ks[r * LDY + tau] = ok ? 1.f : 0.f;
          if (!ok && tau >= M) atomicAdd(&nanc[r], 1);  // rare: gaps (the front padding is in season 0)
        }
      }
    }
  }
  __syncthreads();
  if (n >= a.N) return;  // no barrier below

  const float* row = ys + sr * LDY;
  const float* krow = ks + sr * LDY;
  // nanmean of seasons 0 and 1 over the series' TPC threads (a fixed shuffle tree)
  float s0 = 0.f, k0 = 0.f, s1 = 0.f, k1 = 0.f;
  for (int p = gp; p < M; p += TPC) {
    s0 += row[p];
    k0 += krow[p];
    s1 += row[M + p];
    k1 += krow[M + p];
  }
#pragma unroll
  for (int o = TPC / 2; o > 0; o >>= 1) {
    s0 += __shfl_xor(s0, o, FM_WAVE);
    k0 += __shfl_xor(k0, o, FM_WAVE);
    s1 += __shfl_xor(s1, o, FM_WAVE);
    k1 += __shfl_xor(k1, o, FM_WAVE);
  }
  const float l0 = k0 > 0.f ? s0 / k0 : 0.f;
  const float l1 = k1 > 0.f ? s1 / k1 : 0.f;
  const float b0 = (l1 - l0) / (float)M;

  V c1, c2, g;
  int ci[GPT];
#pragma unroll
  for (int k = 0; k < GPT; ++k) {
    ci[k] = min(GPT * gp + k, a.G - 1);
    const float al = a.grid[3 * ci[k]], be = a.grid[3 * ci[k] + 1], ga = a.grid[3 * ci[k] + 2];
    const float q2 = al * be;
    if constexpr (GPT == 1) {
      c1 = al + q2; c2 = q2; g = ga * (1.f - al);
    } else {
      if (k == 0) { c1.x = al + q2; c2.x = q2; g.x = ga * (1.f - al); }
      else { c1.y = al + q2; c2.y = q2; g.y = ga * (1.f - al); }
    }
  }

  V s[M];  // s[p] = y[p] - l0 (0 where missing)
#pragma unroll
  for (int p = 0; p < M; p += 4) {
    const v4f y4 = *(const v4f*)(row + p);
    const v4f k4 = *(const v4f*)(krow + p);
    s[p + 0] = splat_<V>(y4.x - k4.x * l0);
    s[p + 1] = splat_<V>(y4.y - k4.y * l0);
    s[p + 2] = splat_<V>(y4.z - k4.z * l0);
    s[p + 3] = splat_<V>(y4.w - k4.w * l0);
  }
  V f = splat_<V>(l0 + b0), b = splat_<V>(b0), sse = splat_<V>(0.f);
  const int nv = (nseg - 1) * M - nanc[sr];
  for (int k = 1; k < nseg; ++k) seq_season<M>(row + k * M, krow + k * M, s, f, b, sse, c1, c2, g);

  // argmin over the thread's grid points, then over the series' TPC threads
  float bs = comp_(sse, 0);
  int bi = ci[0];
#pragma unroll
  for (int k = 1; k < GPT; ++k) {
    const float sk = comp_(sse, k);
    if (sk < bs || (sk == bs && ci[k] < bi)) { bs = sk; bi = ci[k]; }
  }
#pragma unroll
  for (int o = TPC / 2; o > 0; o >>= 1) {
    const float os = __shfl_xor(bs, o, FM_WAVE);
    const int oi = __shfl_xor(bi, o, FM_WAVE);
    if (os < bs || (os == bs && oi < bi)) { bs = os; bi = oi; }
  }
  if (gp != bi / GPT) return;  // the winner's owner writes the series' outputs
  const int kw = bi - GPT * gp;
  const float fb = comp_(f, kw), bb = comp_(b, kw);
  a.level[n] = fb - bb;
  a.trend[n] = bb;
  a.sigma[n] = sqrtf(bs / fmaxf((float)nv, 1.f));
  a.best[n] = bi;
  a.nvalid_out[n] = (float)nv;
  float* hb = a.season_hb + (long long)n * SEQ_HB;
#pragma unroll
  for (int p = 0; p < (M < SEQ_HB ? M : SEQ_HB); ++p) hb[p] = comp_(s[p], kw);
  if (a.season_out) {
    float* so = a.season_out + (long long)n * M;
#pragma unroll
    for (int p = 0; p < M; ++p) so[p] = comp_(s[p], kw);
  }
}

// grid points per thread at season M: two (packed) while 2 M VGPRs of season fit beside
// the walk's ~30, else one.  M = 288 (opt-in, kernels.py FOREMAST_HW_SEQ288=1): one grid
// point per thread at one wave per SIMD, 133 of the season's registers in AGPRs; its cost
// does not depend on gaps (5.89 ms per 100k x 2016 x 64 dense or at 1e-3 misses), so it
// beats variant 5 (2.59 dense, 4.78 with 20 % outages, 7.71 at 1e-3 misses) only when most
// series pairs are gapped (profiles/hw_r6/seq/fit_k288_quad_vs_seq.jsonl)
// (A/B: FOREMAST_HW_SEQ_GPT144=2 runs m = 144 with two grid points per thread at one wave
// per SIMD, part of the 288 season registers in AGPRs)
int seq_gpt(int M) {
  if (M <= 96) return 2;
  if (M == 144) {
    const char* e = getenv("FOREMAST_HW_SEQ_GPT144");
    return (e && e[0] == '2') ? 2 : 1;
  }
  return 1;
}

int seq_tpc(int M, int G) {
  const int gpt = seq_gpt(M);
  int t = gpt == 2 ? 16 : 32;  // instantiated: 16 / 32 (two per thread), 32 / 64 (one)
  while (t * gpt < G) t *= 2;
  return t;
}

bool seq_supported_m(int M) { return M == 24 || M == 48 || M == 72 || M == 96 || M == 144 || M == 288; }

template <int M, int GPT, typename TIN>
hipError_t launch_seq(const SmoothArgs& a, int tpc, size_t lds, hipStream_t st) {
  const int sw = 256 / tpc;
  const dim3 grid((a.N + sw - 1) / sw), block(256);
  if constexpr (GPT == 2) {
    if (tpc == 16) hipLaunchKernelGGL((hw_seq_kernel<M, GPT, 16, TIN>), grid, block, lds, st, a);
    else hipLaunchKernelGGL((hw_seq_kernel<M, GPT, 32, TIN>), grid, block, lds, st, a);
  } else {
    if (tpc == 32) hipLaunchKernelGGL((hw_seq_kernel<M, GPT, 32, TIN>), grid, block, lds, st, a);
    else hipLaunchKernelGGL((hw_seq_kernel<M, GPT, 64, TIN>), grid, block, lds, st, a);
  }
  return hipGetLastError();
}

template <typename TIN>
hipError_t launch_seq_m(const SmoothArgs& a, int tpc, size_t lds, hipStream_t st) {
  switch (a.m) {
    case 24: return launch_seq<24, 2, TIN>(a, tpc, lds, st);
    case 48: return launch_seq<48, 2, TIN>(a, tpc, lds, st);
    case 72: return launch_seq<72, 2, TIN>(a, tpc, lds, st);
    case 96: return launch_seq<96, 2, TIN>(a, tpc, lds, st);
    case 144:
      return seq_gpt(144) == 2 ? launch_seq<144, 2, TIN>(a, tpc, lds, st) : launch_seq<144, 1, TIN>(a, tpc, lds, st);
    default: return launch_seq<288, 1, TIN>(a, tpc, lds, st);
  }
}

}  // namespace

// threads per series of the sequential HW fit (0: season not instantiated or G out of range)
extern "C" int fm_hw_seq_tpc(int m, int G) {
  if (!seq_supported_m(m) || G < 1 || G > 64) return 0;
  return seq_tpc(m, G);
}

// LDS bytes of one workgroup ((size_t)-1: unsupported season / grid / length)
extern "C" size_t fm_hw_seq_lds_bytes(int Tp, int m, int G) {
  const int tpc = fm_hw_seq_tpc(m, G);
  if (tpc == 0 || Tp % m != 0 || Tp / m < 2) return (size_t)-1;
  const int sw = 256 / tpc;
  return ((size_t)2 * sw * (Tp + 4) + (size_t)sw) * 4;
}

// Holt-Winters grid fit at a short season (m in 24 / 48 / 72 / 96 / 144), plus the band /
// verdict epilogue when det.C > 0.  Needs level, trend, sigma, best, nvalid_out and
// season_hb [N, 16]; season_out [N, m] optional.  T <= ring_len, Tp = ceil(T / m) m,
// pad = Tp - T; head from head_dev when set (HIP-graph replays).
extern "C" int fm_hw_seq_fit(const SmoothArgs* a, int bf16, hipStream_t st) {
  if (a->N <= 0) return 0;
  const int m = a->m;
  const size_t lds = fm_hw_seq_lds_bytes(a->Tp, m, a->G);
  if (lds == (size_t)-1 || lds > 64 * 1024) return (int)hipErrorNotSupported;
  if (a->T < 1 || a->T > a->ring_len || a->pad != a->Tp - a->T || a->pad < 0 || a->pad >= m ||
      (!a->head_dev && (a->head < 0 || a->head >= a->ring_len)) || a->ld < a->ring_len || !a->grid ||
      !a->level || !a->trend || !a->sigma || !a->best || !a->nvalid_out || !a->season_hb)
    return (int)hipErrorInvalidValue;
  const int tpc = seq_tpc(m, a->G);
  const hipError_t e = bf16 ? launch_seq_m<bf16_t>(*a, tpc, lds, st) : launch_seq_m<float>(*a, tpc, lds, st);
  if (e != hipSuccess) return (int)e;
  if (a->det.C <= 0) return 0;
  return fm_hw_detect_params(a, st);
}
