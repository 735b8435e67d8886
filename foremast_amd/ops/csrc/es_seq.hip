// K2 sequential form: exponential / double exponential smoothing grid fit with one
// (series, pair of grid points) per thread.
//
// Same semantics as models/smoothing.py (MODE_ES / MODE_DES): l0 = first valid value,
// b0 = 0, error-correction updates l <- l + b + alpha e, b <- b + alpha beta e, missing
// points imputed by the forecast (e = 0) and excluded from the SSE, argmin SSE over the
// grid (lowest index on ties), sigma = sqrt(SSE / n_valid).
//
// Why not the time-parallel scan of hw_scan.hip: ES / DES carry a 1- or 2-float state,
// so N x G independent chains (100k series x 4..16 grid points) already fill the chip;
// walking them sequentially costs 3 (ES) or 6 (DES) packed FP32 ops per step for two
// grid points, against a scan's per-segment composition and carry passes.  The work
// is staged through LDS: a workgroup owns 256 / tpc series (tpc = threads per series),
// loads 64-step chunks of all its rows with coalesced 128-byte row segments into a
// double-buffered [series][65] fp32 tile (row stride 65: the series of a wave hit
// distinct banks), and every thread walks its row from LDS while the next chunk's loads
// are in flight.  Chunks with a missing point take a masked walk; the rest are
// straight-line.  The band / verdict epilogue is fm_hw_detect_params with m = 1.
#include "common.h"
#include "args.h"

extern __shared__ __attribute__((aligned(16))) char fm_es_smem[];

extern "C" int fm_hw_detect_params(const SmoothArgs* a, hipStream_t st);

namespace {

constexpr int ES_TC = 64;
constexpr int ES_LD = ES_TC + 1;
enum { MODE_ES = 0, MODE_DES = 1 };

template <int MODE, bool SAFE>
__device__ __forceinline__ void es_walk(const float* row, int nt, v2f al, v2f c2, v2f& l, v2f& b, v2f& sse,
                                        bool& started) {
#pragma unroll 8
  for (int t = 0; t < nt; ++t) {
    const float y = row[t];
    v2f e;
    if (SAFE) {
      const bool ok = y == y;
      if (ok && !started) {  // first valid point: l0 = y (e = 0 there)
        l = splat2(y);
        started = true;
      }
      e = splat2(ok ? y : 0.f) - l;
      if (MODE == MODE_DES) e = e - b;
      e = ok ? e : splat2(0.f);
    } else {
      e = splat2(y) - l;
      if (MODE == MODE_DES) e = e - b;
    }
    if (MODE == MODE_ES) {
      l = l + al * e;
    } else {
      const v2f f = l + b;
      l = f + al * e;
      b = b + c2 * e;
    }
    sse = sse + e * e;
  }
}

template <int MODE, typename TIN, int TPC>
__global__ __launch_bounds__(256) void es_seq_kernel(const SmoothArgs a) {
  constexpr int SW = 256 / TPC;             // series per workgroup
  constexpr int PER = SW * ES_TC / 256;     // staged elements per thread per chunk
  const int tid = threadIdx.x;
  const int s = tid / TPC, gp = tid - s * TPC;
  const int n0 = blockIdx.x * SW;
  const int n = n0 + s;
  float* tile = (float*)fm_es_smem;               // [2][SW][ES_LD]
  int* nanc = (int*)(tile + 2 * SW * ES_LD);      // [2][SW]  missing points per chunk
  const int T = a.T, R = a.ring_len;
  const int nch = (T + ES_TC - 1) / ES_TC;
  const TIN* base = (const TIN*)a.hist;

  const int c0 = min(2 * gp, a.G - 1), c1 = min(2 * gp + 1, a.G - 1);
  v2f al, be;
  al.x = a.grid[3 * c0]; al.y = a.grid[3 * c1];
  be.x = a.grid[3 * c0 + 1]; be.y = a.grid[3 * c1 + 1];
  const v2f c2 = al * be;

  float v[PER];
  // loads of chunk ch into registers: element e = tid + 256 k -> (row e / 64, step e % 64),
  // so a wave reads one 128-byte row segment per load; rows / steps out of range read a
  // clamped valid column and become 0 (not NaN: they are never walked nor counted)
  auto load_chunk = [&](int ch) {
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int e = tid + 256 * k, se = e / ES_TC, t = ch * ES_TC + (e % ES_TC);
      const bool ok = (n0 + se < a.N) && (t < T);
      int c = a.head + (ok ? t : 0);
      c -= (c >= R) ? R : 0;
      const float x = to_f32<TIN>(base[(long long)(ok ? n0 + se : 0) * a.ld + c]);
      v[k] = ok ? x : 0.f;
    }
  };
  auto store_chunk = [&](int buf) {
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int e = tid + 256 * k, se = e / ES_TC, t = e % ES_TC;
      tile[(buf * SW + se) * ES_LD + t] = v[k];
      if (v[k] != v[k]) atomicAdd(&nanc[buf * SW + se], 1);
    }
  };

  for (int i = tid; i < 2 * SW; i += blockDim.x) nanc[i] = 0;
  __syncthreads();
  load_chunk(0);
  store_chunk(0);
  __syncthreads();

  v2f l = splat2(0.f), b = splat2(0.f), sse = splat2(0.f);
  bool started = false;
  int nv = 0;
  for (int ch = 0; ch < nch; ++ch) {
    const int buf = ch & 1;
    const bool more = ch + 1 < nch;
    if (more) load_chunk(ch + 1);                   // in flight during the walk
    if (more && tid < SW) nanc[(buf ^ 1) * SW + tid] = 0;
    const int nt = min(ES_TC, T - ch * ES_TC);
    const float* row = tile + (buf * SW + s) * ES_LD;
    const int miss = nanc[buf * SW + s];
    nv += nt - miss;
    if (miss == 0 && !started) {
      l = splat2(row[0]);
      started = true;
    }
    if (__all(miss == 0)) es_walk<MODE, false>(row, nt, al, c2, l, b, sse, started);
    else es_walk<MODE, true>(row, nt, al, c2, l, b, sse, started);
    __syncthreads();                                // buf^1 free, its counters zeroed
    if (more) store_chunk(buf ^ 1);
    __syncthreads();
  }

  // argmin over this thread's two grid points, then over the TPC threads of the series
  float bs = sse.x, bl = l.x, bb = b.x;
  int bi = c0;
  if (sse.y < bs || (sse.y == bs && c1 < bi)) { bs = sse.y; bl = l.y; bb = b.y; bi = c1; }
#pragma unroll
  for (int o = TPC / 2; o > 0; o >>= 1) {
    const float os = __shfl_xor(bs, o, FM_WAVE), ol = __shfl_xor(bl, o, FM_WAVE), ob = __shfl_xor(bb, o, FM_WAVE);
    const int oi = __shfl_xor(bi, o, FM_WAVE);
    if (os < bs || (os == bs && oi < bi)) { bs = os; bl = ol; bb = ob; bi = oi; }
  }
  if (gp == 0 && n < a.N) {
    a.level[n] = bl;
    a.trend[n] = bb;
    a.sigma[n] = sqrtf(bs / fmaxf((float)nv, 1.f));
    a.best[n] = bi;
    a.nvalid_out[n] = (float)nv;
  }
}

template <int MODE, typename TIN>
hipError_t launch_es(const SmoothArgs& a, int tpc, hipStream_t st) {
  const int sw = 256 / tpc;
  const size_t lds = (size_t)2 * sw * ES_LD * 4 + (size_t)2 * sw * 4;
  const dim3 grid((a.N + sw - 1) / sw), block(256);
  switch (tpc) {
    case 1: hipLaunchKernelGGL((es_seq_kernel<MODE, TIN, 1>), grid, block, lds, st, a); break;
    case 2: hipLaunchKernelGGL((es_seq_kernel<MODE, TIN, 2>), grid, block, lds, st, a); break;
    case 4: hipLaunchKernelGGL((es_seq_kernel<MODE, TIN, 4>), grid, block, lds, st, a); break;
    case 8: hipLaunchKernelGGL((es_seq_kernel<MODE, TIN, 8>), grid, block, lds, st, a); break;
    case 16: hipLaunchKernelGGL((es_seq_kernel<MODE, TIN, 16>), grid, block, lds, st, a); break;
    default: hipLaunchKernelGGL((es_seq_kernel<MODE, TIN, 32>), grid, block, lds, st, a); break;
  }
  return hipGetLastError();
}

}  // namespace

// threads per series for a grid of G points (two per thread), a power of two <= 32
extern "C" int fm_es_seq_tpc(int G) {
  int t = 1;
  while (2 * t < G) t *= 2;
  return t;
}

// ES / DES grid fit (+ the detection epilogue when det.C > 0).  Needs level, trend,
// sigma, best, nvalid_out and (for the epilogue) a zeroed season_hb [N, 16]; T <= R.
extern "C" int fm_es_seq_fit(const SmoothArgs* a, int mode, int bf16, hipStream_t st) {
  if (a->N <= 0) return 0;
  if ((mode != MODE_ES && mode != MODE_DES) || a->G < 1 || a->G > 64 || a->T < 1 || a->T > a->ring_len ||
      a->head < 0 || a->head >= a->ring_len || !a->nvalid_out || !a->level || !a->trend || !a->sigma || !a->best)
    return (int)hipErrorInvalidValue;
  const int tpc = fm_es_seq_tpc(a->G);
  hipError_t e;
  if (mode == MODE_ES)
    e = bf16 ? launch_es<MODE_ES, bf16_t>(*a, tpc, st) : launch_es<MODE_ES, float>(*a, tpc, st);
  else
    e = bf16 ? launch_es<MODE_DES, bf16_t>(*a, tpc, st) : launch_es<MODE_DES, float>(*a, tpc, st);
  if (e != hipSuccess) return (int)e;
  if (a->det.C <= 0) return 0;
  SmoothArgs d = *a;
  d.Tp = a->T;
  d.m = 1;
  return fm_hw_detect_params(&d, st);
}
