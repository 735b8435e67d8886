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
// walking them sequentially costs 3 (ES) or 5 (DES) packed FP32 ops per step for two
// grid points, against a scan's per-segment composition and carry passes.  The work
// is staged through LDS: a workgroup owns 256 / tpc series (tpc = threads per series),
// loads 64-step chunks of all its rows with coalesced 128-byte row segments into a
// [series][65] fp32 tile (row stride 65: the series of a wave hit distinct banks), and
// every thread walks its row from LDS while the next two chunks load into registers
// (loads are issued unconditionally, clamped to the last chunk, so the wait before a
// store covers only the older chunk).  The tile is single-buffered so that four
// 128-series workgroups fit a CU: the 100k-series ES grid is one round of workgroups.
// A chunk's missing points are counted with one ballot per row; chunks with a missing
// point take a masked walk, the rest are straight-line.  The
// band / verdict epilogue is fm_hw_detect_params with m = 1.
#include "common.h"
#include "args.h"

extern __shared__ __attribute__((aligned(16))) char fm_es_smem[];

extern "C" int fm_hw_detect_params(const SmoothArgs* a, hipStream_t st);

namespace {

constexpr int ES_TC = 64;
constexpr int ES_LD = ES_TC + 1;
static_assert(ES_TC == FM_WAVE, "one wave-wide load is one row's chunk (missing counts by ballot)");
enum { MODE_ES = 0, MODE_DES = 1 };
constexpr int FM_BUF_DW3 = 0x00020000;  // buffer resource word 3 (raw dword access) on gfx950

// raw bits of one element (bf16: zero-extended 16 bits); converted when stored to LDS so
// that nothing waits on the load before then
template <typename TIN>
__device__ __forceinline__ unsigned buf_load(__amdgpu_buffer_rsrc_t r, unsigned off, unsigned soff) {
  if (sizeof(TIN) == 2) return (unsigned)__builtin_amdgcn_raw_buffer_load_b16(r, off, soff, 0);
  return __builtin_amdgcn_raw_buffer_load_b32(r, off, soff, 0);
}
template <typename TIN>
__device__ __forceinline__ float bits_f32(unsigned u) {
  return __uint_as_float(sizeof(TIN) == 2 ? u << 16 : u);
}

template <int MODE, bool SAFE>
__device__ __forceinline__ void es_walk(const float* row, int nt, v2f al, v2f c2, v2f& l, v2f& b, v2f& sse,
                                        bool& started) {
#pragma unroll 8
  for (int t = 0; t < nt; ++t) {
    const float y = row[t];
    v2f e, f;
    if (MODE == MODE_DES) f = l + b;  // one-step forecast
    if (SAFE) {
      const bool ok = y == y;
      if (ok && !started) {  // first valid point: l0 = y (e = 0 there)
        l = splat2(y);
        if (MODE == MODE_DES) f = l + b;
        started = true;
      }
      e = splat2(ok ? y : 0.f) - (MODE == MODE_DES ? f : l);
      e = ok ? e : splat2(0.f);
    } else {
      e = splat2(y) - (MODE == MODE_DES ? f : l);
    }
    if (MODE == MODE_ES) {
      l = l + al * e;
    } else {
      l = f + al * e;
      b = b + c2 * e;
    }
    sse = sse + e * e;
  }
}

// PARTIAL: N < SW (one workgroup with rows past N).  Otherwise every workgroup owns SW
// valid rows: the last one is shifted back to N - SW and recomputes (bit-identically)
// some series of its neighbour.
template <int MODE, typename TIN, int TPC, bool PARTIAL>
__global__ __launch_bounds__(256) void es_seq_kernel(const SmoothArgs a) {
  constexpr int SW = 256 / TPC;             // series per workgroup
  constexpr int PER = SW * ES_TC / 256;     // staged elements per thread per chunk
  // double-buffered tile (one barrier per chunk) when it stays small: <= 64 series, 33 KB;
  // the 128-series single tile keeps four workgroups on a CU
  constexpr int NB = SW <= 64 ? 2 : 1;
  const int tid = threadIdx.x;
  const int s = tid / TPC, gp = tid - s * TPC;
  const int n0 = PARTIAL ? 0 : min((int)blockIdx.x * SW, a.N - SW);
  const int n = n0 + s;
  float* tiles = (float*)fm_es_smem;              // [NB][SW][ES_LD]  chunks (walked / being staged)
  int* nancs = (int*)(tiles + NB * SW * ES_LD);   // [NB][SW]         missing points of each chunk
  const int T = a.T, R = a.ring_len;
  const int nch = (T + ES_TC - 1) / ES_TC;
  const TIN* base = (const TIN*)a.hist;

  const int c0 = min(2 * gp, a.G - 1), c1 = min(2 * gp + 1, a.G - 1);
  v2f al, be;
  al.x = a.grid[3 * c0]; al.y = a.grid[3 * c1];
  be.x = a.grid[3 * c0 + 1]; be.y = a.grid[3 * c1 + 1];
  const v2f c2 = al * be;

  // loads of chunk ch (clamped to the last one) into registers: element e = tid + 256 k
  // -> (row e / 64, step e % 64), so a wave reads one 128-byte row segment per load.
  // A raw buffer over this workgroup's rows gives one 32-bit lane offset per element
  // (no 64-bit address per element), and rows past N read 0 through the hardware range
  // check; steps past T read a valid column
  const int nrow = min(SW, a.N - n0);
  const __amdgpu_buffer_rsrc_t rows = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(base + (long long)n0 * a.ld), (short)0, (int)(nrow * a.ld * (long long)sizeof(TIN)), FM_BUF_DW3);
  const unsigned row_step = (unsigned)(256 / ES_TC) * (unsigned)a.ld * (unsigned)sizeof(TIN);
  auto load_chunk = [&](int ch, unsigned (&v)[PER]) {
    ch = min(ch, nch - 1);
    const int t = ch * ES_TC + (tid % ES_TC);  // the same step for every k (256 % ES_TC == 0)
    int c = a.head + (t < T ? t : 0);
    c -= (c >= R) ? R : 0;
    const unsigned vo = (unsigned)((tid / ES_TC) * (int)a.ld + c) * (unsigned)sizeof(TIN);
    if (!PARTIAL) {  // every row in range: the per-row step rides in the scalar offset
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        v[k] = buf_load<TIN>(rows, vo, (unsigned)k * row_step);
      }
    } else {         // N < SW: rows past N read 0 through the range-checked lane offset
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        v[k] = buf_load<TIN>(rows, vo + (unsigned)k * row_step, 0u);
      }
    }
  };
  // chunk ch into the tile; steps past T become 0 (not NaN: never walked or counted)
  auto store_chunk = [&](int ch, const unsigned (&v)[PER]) {
    float* tile = tiles + (ch % NB) * SW * ES_LD;
    int* nanc = nancs + (ch % NB) * SW;
    const int t = tid % ES_TC;
    const bool okt = ch * ES_TC + t < T;
    // the missing count of load k (row se's whole chunk: one ballot) goes to lane k of one
    // register (v_writelane), and lanes 0..PER-1 store them once: no single-lane LDS store
    // and exec-mask round trip per row
    int cnt = 0;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int se = tid / ES_TC + k * (256 / ES_TC);
      const float x = okt ? bits_f32<TIN>(v[k]) : 0.f;
      tile[se * ES_LD + t] = x;
      const int miss = __popcll(__ballot(x != x));  // wave-uniform (an SGPR)
      asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(cnt) : "s"(miss), "i"(k));
    }
    if (t < PER) nanc[tid / ES_TC + t * (256 / ES_TC)] = cnt;
  };

  unsigned va[PER], vb[PER];
  load_chunk(0, va);
  store_chunk(0, va);
  load_chunk(1, va);
  __syncthreads();

  v2f l = splat2(0.f), b = splat2(0.f), sse = splat2(0.f);
  bool started = false;
  int nv = 0;
  // walk chunk ch from its tile while nx (chunk ch + 1) and pf (chunk ch + 2) load
  auto body = [&](int ch, unsigned (&nx)[PER], unsigned (&pf)[PER]) {
    load_chunk(ch + 2, pf);
    // double-buffered: chunk ch + 1 goes to the other tile now (its last reader, the walk
    // of chunk ch - 1, finished before the previous barrier)
    if (NB == 2 && ch + 1 < nch) store_chunk(ch + 1, nx);
    const float* row = tiles + (ch % NB) * SW * ES_LD + s * ES_LD;
    const int nt = min(ES_TC, T - ch * ES_TC);
    const int miss = nancs[(ch % NB) * SW + s];
    nv += nt - miss;
    if (miss == 0 && !started) {
      l = splat2(row[0]);
      started = true;
    }
    if (__all(miss == 0)) es_walk<MODE, false>(row, nt, al, c2, l, b, sse, started);
    else es_walk<MODE, true>(row, nt, al, c2, l, b, sse, started);
    __syncthreads();                                // tile and counts free (NB = 2: chunk ch + 1 staged)
    if (NB == 1) {
      if (ch + 1 < nch) store_chunk(ch + 1, nx);
      __syncthreads();
    }
  };
  for (int ch = 0; ch < nch; ch += 2) {
    body(ch, va, vb);
    if (ch + 1 < nch) body(ch + 1, vb, va);
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
  const int nb = sw <= 64 ? 2 : 1;  // the kernel's NB
  const size_t lds = (size_t)nb * sw * ES_LD * 4 + (size_t)nb * sw * 4;
  const dim3 grid((a.N + sw - 1) / sw), block(256);
  if (a.N < sw) {
    switch (tpc) {
      case 1: hipLaunchKernelGGL((es_seq_kernel<MODE, TIN, 1, true>), grid, block, lds, st, a); break;
      case 2: hipLaunchKernelGGL((es_seq_kernel<MODE, TIN, 2, true>), grid, block, lds, st, a); break;
      case 4: hipLaunchKernelGGL((es_seq_kernel<MODE, TIN, 4, true>), grid, block, lds, st, a); break;
      case 8: hipLaunchKernelGGL((es_seq_kernel<MODE, TIN, 8, true>), grid, block, lds, st, a); break;
      case 16: hipLaunchKernelGGL((es_seq_kernel<MODE, TIN, 16, true>), grid, block, lds, st, a); break;
      default: hipLaunchKernelGGL((es_seq_kernel<MODE, TIN, 32, true>), grid, block, lds, st, a); break;
    }
    return hipGetLastError();
  }
  switch (tpc) {
    case 1: hipLaunchKernelGGL((es_seq_kernel<MODE, TIN, 1, false>), grid, block, lds, st, a); break;
    case 2: hipLaunchKernelGGL((es_seq_kernel<MODE, TIN, 2, false>), grid, block, lds, st, a); break;
    case 4: hipLaunchKernelGGL((es_seq_kernel<MODE, TIN, 4, false>), grid, block, lds, st, a); break;
    case 8: hipLaunchKernelGGL((es_seq_kernel<MODE, TIN, 8, false>), grid, block, lds, st, a); break;
    case 16: hipLaunchKernelGGL((es_seq_kernel<MODE, TIN, 16, false>), grid, block, lds, st, a); break;
    default: hipLaunchKernelGGL((es_seq_kernel<MODE, TIN, 32, false>), grid, block, lds, st, a); break;
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
      a->head < 0 || a->head >= a->ring_len || a->ld < a->ring_len || a->ld > (1 << 20) || !a->nvalid_out || !a->level || !a->trend || !a->sigma || !a->best)
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
