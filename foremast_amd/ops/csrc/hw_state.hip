// Cached Holt-Winters model (K3 state): extract the full state of the fitted model once
// per refit, then advance it by the newly graduated points and score the current window
// on every tick in between, in O(1) per series instead of an O(T x G) refit.
//
// The reference brain keeps fitted models in an LRU cache (MAX_CACHE_SIZE,
// foremast-brain/README.md:30) instead of refitting on every request; this is the
// streaming engine's equivalent.  Semantics: models/smoothing.py (hw_run, hw_update):
//
//   refit tick:  the grid fit picks (alpha, beta, gamma) per series (hw_scan.hip); this
//                file's hw_state_kernel re-walks the window with THAT grid point and
//                keeps level, trend and all m seasonal terms (one thread per series);
//   other ticks: hw_update_detect_kernel applies the same error-correction update to the
//                graduated point(s), then forecasts the current window from the state and
//                runs the shared band / verdict epilogue (detect.h) with the refit's
//                sigma, valid count and grid index (h-step variance).
//
// Layout: the seasonal state is phase-major, season[p * N + n], so the 64 series of a
// wave read and write one contiguous 256-byte segment per step in both kernels.
//
// hw_state_kernel stages the history like es_seq.hip: a workgroup of 128 threads owns
// 128 series and loads 64-step chunks with coalesced 128-byte row segments into a
// [series][65] fp32 LDS tile, one chunk ahead of the walk.
#include "common.h"
#include "args.h"
#include "detect.h"

struct HwStateArgs {
  const void* hist;   // [N, ld] ring (float or bf16)
  long long ld;
  int ring_len;
  int head;           // physical column of logical t = 0
  int T;              // logical window length
  int Tp;             // padded length (multiple of m; the first pad steps are missing)
  int m;
  int N;
  int bf16;
  int _pad0;
  const float* grid;  // [G, 3]
  const int* best;    // [N] grid index chosen by the fit
  float* level;       // [N]
  float* trend;       // [N]
  float* season;      // [m, N] phase-major
  float* nvalid;      // [N] valid points the fit counted (padded steps m .. Tp-1)
};

struct HwUpdateArgs {
  const void* hist;     // [N, ld] ring (float or bf16)
  long long ld;
  int ring_len;
  int col0;             // physical column of the first new point
  int npts;             // new points to apply (columns col0 .. col0 + npts - 1, mod R)
  int t_last;           // padded time of the last point already in the state
  int m;
  int N;
  int bf16;
  int _pad0;
  const float* grid;    // [G, 3]
  const int* best;      // [N]
  float* level;         // [N]
  float* trend;         // [N]
  float* season;        // [m, N]
  const float* sigma;   // [N] residual std of the refit
  const float* nvalid;  // [N] valid points of the refit window
  DetectArgs det;
};

extern __shared__ __attribute__((aligned(16))) char fm_hws_smem[];

namespace {

constexpr int HS_SW = 128;   // series (= threads) per workgroup
constexpr int HS_TC = 64;    // steps per staged chunk
constexpr int HS_LD = HS_TC + 1;
constexpr int HS_BUF_DW3 = 0x00020000;  // buffer resource word 3 (raw dword access) on gfx950
static_assert(HS_TC == FM_WAVE, "a wave-wide load is one row's chunk");

template <typename TIN>
__device__ __forceinline__ float ld_hist(const TIN* base, long long ld, int row, int col) {
  return to_f32<TIN>(base[(long long)row * ld + col]);
}

// One thread per series.  Software pipeline per 64-step chunk: the next chunk's history
// is loaded into registers (hv) while the current one is walked from the LDS tile, and
// each seasonal term is re-loaded for the next chunk right after its last use in this
// one (phase p + 64: never a phase this chunk still writes, as m >= 128), so neither
// load waits on the walk.
template <typename TIN>
__global__ __launch_bounds__(HS_SW) void hw_state_kernel(const HwStateArgs a) {
  const int tid = threadIdx.x;
  const int n0 = blockIdx.x * HS_SW;
  const int n = n0 + tid;
  const bool live = n < a.N;
  float* tile = (float*)fm_hws_smem;  // [HS_SW][HS_LD]
  const TIN* base = (const TIN*)a.hist;
  const int T = a.T, R = a.ring_len, m = a.m, N = a.N, Tp = a.Tp;
  const int pad = Tp - T;
  const int nrow = min(HS_SW, N - n0);
  const int lane = lane_id(), wv = wave_id();
  constexpr int RPW = HS_SW / (HS_SW / FM_WAVE);  // rows staged per wave (64): row = wv + 2 i

  // history of padded steps [tp0, tp0 + 64) of this wave's rows (lane = step) through a
  // raw buffer over the workgroup's rows: one 32-bit lane offset, the row step rides in
  // the scalar offset, rows past N read 0 through the range check (not live)
  const __amdgpu_buffer_rsrc_t rows = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(base + (long long)n0 * a.ld), (short)0, (int)(nrow * a.ld * (long long)sizeof(TIN)), HS_BUF_DW3);
  const unsigned row_step = 2u * (unsigned)a.ld * (unsigned)sizeof(TIN);
  // raw bits in flight; converted (and out-of-window steps set to NaN) when stored to
  // LDS, so nothing waits on a load before the next chunk's store
  unsigned hv[RPW];
  bool hok = false;
  auto load = [&](int tp0) {
    const int t = tp0 + lane - pad;
    hok = t >= 0 && t < T && tp0 + lane < Tp;
    int c = a.head + (hok ? t : 0);
    c -= (c >= R) ? R : 0;
    const unsigned vo = (unsigned)(wv * (int)a.ld + c) * (unsigned)sizeof(TIN);
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      if (sizeof(TIN) == 2) hv[i] = (unsigned)__builtin_amdgcn_raw_buffer_load_b16(rows, vo, (unsigned)i * row_step, 0);
      else hv[i] = __builtin_amdgcn_raw_buffer_load_b32(rows, vo, (unsigned)i * row_step, 0);
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      const float x = __uint_as_float(sizeof(TIN) == 2 ? hv[i] << 16 : hv[i]);
      tile[(wv + 2 * i) * HS_LD + lane] = hok ? x : fm_nan();
    }
  };

  float al = 0.f, ab = 0.f, g1a = 0.f;
  if (live) {
    const int gi = a.best[n];
    al = a.grid[3 * gi];
    ab = al * a.grid[3 * gi + 1];
    g1a = a.grid[3 * gi + 2] * (1.f - al);
  }
  const float* row = tile + tid * HS_LD;
  // seasonal state through a raw buffer: the phase is wave-uniform, so a step's address
  // is the lane's fixed series offset plus a scalar phase offset (p * N * 4 < 2^31, host
  // check); threads past N access past the buffer's range (dropped)
  const __amdgpu_buffer_rsrc_t seab = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.season, (short)0, (int)((long long)m * N * 4), HS_BUF_DW3);
  const unsigned so_n = live ? (unsigned)n * 4u : 0x7ffffff0u;
  const unsigned pstride = (unsigned)N * 4u;
  auto sea_ld = [&](int p) { return __builtin_amdgcn_raw_buffer_load_b32(seab, so_n, (unsigned)p * pstride, 0); };
  auto sea_st = [&](int p, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), seab, so_n, (unsigned)p * pstride, 0);
  };

  // Chunks of [t0, t1) walked from the tile while the next chunk loads: full chunks run
  // `full` (straight-line, unrolled), a last partial one runs `part`; every load is
  // unconditional (out-of-window steps read NaN) so no wait depends on a branch.
  auto chunks = [&](int t0, int t1, auto&& full, auto&& part) {
    load(t0);
    for (int tp0 = t0; tp0 < t1; tp0 += HS_TC) {
      __syncthreads();
      store();
      __syncthreads();
      load(tp0 + HS_TC);
      if (tp0 + HS_TC <= t1) full(tp0);
      else part(tp0, t1 - tp0);
    }
  };

  // pass 1: season 0 (raw values into the state, NaN kept, and its mean), season 1 (mean)
  float s0 = 0.f, s1 = 0.f;
  int c0 = 0, c1 = 0;
  chunks(0, m, [&](int tp0) {
#pragma unroll
    for (int j = 0; j < HS_TC; ++j) {
      const float y = row[j];
      sea_st(tp0 + j, y);
      s0 += (y == y) ? y : 0.f;
      c0 += (y == y);
    }
  }, [&](int tp0, int nt) {
    for (int j = 0; j < nt; ++j) {
      const float y = row[j];
      sea_st(tp0 + j, y);
      s0 += (y == y) ? y : 0.f;
      c0 += (y == y);
    }
  });
  auto acc1 = [&](int nt) {
    for (int j = 0; j < nt; ++j) {
      const float y = row[j];
      s1 += (y == y) ? y : 0.f;
      c1 += (y == y);
    }
  };
  chunks(m, 2 * m, [&](int) { acc1(HS_TC); }, [&](int, int nt) { acc1(nt); });
  const float l0 = c0 > 0 ? s0 / (float)c0 : 0.f;
  const float l1 = c1 > 0 ? s1 / (float)c1 : 0.f;
  float lvl = l0, trd = (l1 - l0) / (float)m;

  // pass 2: the error-correction recursion over padded steps m .. Tp-1; a phase's state
  // is first read in season 1, where the raw season-0 value becomes y - l0 (0 if missing).
  // sv[j] holds the term of step j of the current chunk; right after its use it is
  // re-loaded for step j of the next chunk (phase + 64)
  float sv[HS_TC];
#pragma unroll
  for (int j = 0; j < HS_TC; ++j) sv[j] = __uint_as_float(sea_ld(j));
  int p0 = 0;  // phase of the chunk's first step
  int nv = 0;
  auto step = [&](int j, int tp, int p, int pn, bool first) {
    float s = sv[j];
    if (first) s = (tp < 2 * m) ? ((s == s) ? s - l0 : 0.f) : s;
    const float y = row[j];
    nv += (y == y);
    const float e = (y == y) ? y - s - lvl - trd : 0.f;
    lvl = lvl + trd + al * e;
    trd = trd + ab * e;
    sea_st(p, s + g1a * e);
    sv[j] = __uint_as_float(sea_ld(pn));
  };
  chunks(m, Tp, [&](int tp0) {
    int p = p0, pn = p0 + HS_TC;
    pn -= (pn >= m) ? m : 0;
    if (tp0 < 2 * m) {
#pragma unroll
      for (int j = 0; j < HS_TC; ++j) {
        step(j, tp0 + j, p, pn, true);
        p = (p + 1 == m) ? 0 : p + 1;
        pn = (pn + 1 == m) ? 0 : pn + 1;
      }
    } else {
#pragma unroll
      for (int j = 0; j < HS_TC; ++j) {
        step(j, tp0 + j, p, pn, false);
        p = (p + 1 == m) ? 0 : p + 1;
        pn = (pn + 1 == m) ? 0 : pn + 1;
      }
    }
    p0 = p;
  }, [&](int tp0, int nt) {
    int p = p0;
#pragma unroll
    for (int j = 0; j < HS_TC; ++j) {
      if (j < nt) {
        float s = sv[j];
        if (tp0 + j < 2 * m) s = (s == s) ? s - l0 : 0.f;
        const float y = row[j];
        nv += (y == y);
        const float e = (y == y) ? y - s - lvl - trd : 0.f;
        lvl = lvl + trd + al * e;
        trd = trd + ab * e;
        sea_st(p, s + g1a * e);
        p = (p + 1 == m) ? 0 : p + 1;
      }
    }
  });
  if (live) {
    a.level[n] = lvl;
    a.trend[n] = trd;
    a.nvalid[n] = (float)nv;
  }
}

template <typename TIN>
__global__ __launch_bounds__(256) void hw_update_detect_kernel(const HwUpdateArgs a) {
  const int n = blockIdx.x * 16 + (threadIdx.x >> 4);  // one 16-lane row per series
  if (n >= a.N) return;  // row-uniform
  const int N = a.N, m = a.m, R = a.ring_len;
  const int gi = a.best[n];
  const float al = a.grid[3 * gi];
  const float ab = al * a.grid[3 * gi + 1];
  const float g1a = a.grid[3 * gi + 2] * (1.f - al);
  float lvl = a.level[n], trd = a.trend[n];
  int t = a.t_last;
  const TIN* base = (const TIN*)a.hist;
  // every lane of the row runs the (scalar) update on the same values; its first stores the state
  for (int k = 0; k < a.npts; ++k) {
    ++t;
    const int p = t % m;
    int c = a.col0 + k;
    c -= (c >= R) ? R : 0;
    const float y = ld_hist<TIN>(base, a.ld, n, c);
    float* sp = a.season + (long long)p * N + n;
    const float s = *sp;
    const float e = (y == y) ? y - s - lvl - trd : 0.f;
    lvl = lvl + trd + al * e;
    trd = trd + ab * e;
    if ((lane_id() & 15) == 0) *sp = s + g1a * e;
  }
  if ((lane_id() & 15) == 0) {
    a.level[n] = lvl;
    a.trend[n] = trd;
  }
  const float* sn = a.season + n;
  detect_epilogue_row(a.det, n, a.sigma[n], a.nvalid[n], [&](int h) {
    return lvl + (float)h * trd + sn[(long long)((t + h) % m) * N];
  }, gi);
}

}  // namespace

extern "C" long long fm_hw_state_args_size() { return (long long)sizeof(HwStateArgs); }
extern "C" long long fm_hw_update_args_size() { return (long long)sizeof(HwUpdateArgs); }

extern "C" size_t fm_hw_state_lds_bytes() { return (size_t)HS_SW * HS_LD * sizeof(float); }

// State of the fitted model (level, trend, season [m, N]) at the end of the window.
extern "C" int fm_hw_state(const HwStateArgs* a, hipStream_t st) {
  if (a->N <= 0) return 0;
  if (a->m < 1 || a->Tp % a->m != 0 || a->Tp / a->m < 2 || a->T < 1 || a->T > a->Tp || a->T > a->ring_len ||
      a->head < 0 || a->head >= a->ring_len || a->ld < a->ring_len || !a->grid || !a->best || !a->level ||
      !a->trend || !a->season || !a->nvalid || a->m < 2 * HS_TC || (long long)a->m * a->N * 4 >= (1ll << 31))
    return (int)hipErrorInvalidValue;
  const dim3 grid((a->N + HS_SW - 1) / HS_SW), block(HS_SW);
  const size_t lds = fm_hw_state_lds_bytes();
  if (a->bf16)
    hipLaunchKernelGGL(hw_state_kernel<bf16_t>, grid, block, lds, st, *a);
  else
    hipLaunchKernelGGL(hw_state_kernel<float>, grid, block, lds, st, *a);
  return (int)hipGetLastError();
}

// Advance the state by npts graduated points and score the current window.
extern "C" int fm_hw_update_detect(const HwUpdateArgs* a, hipStream_t st) {
  if (a->N <= 0) return 0;
  if (a->m < 1 || a->npts < 0 || a->npts > a->ring_len || a->col0 < 0 || a->col0 >= a->ring_len ||
      a->t_last < 0 || a->ld < a->ring_len || !a->grid || !a->best || !a->level || !a->trend || !a->season ||
      !a->sigma || !a->nvalid)
    return (int)hipErrorInvalidValue;
  const dim3 grid((a->N + 15) / 16), block(256);
  if (a->bf16)
    hipLaunchKernelGGL(hw_update_detect_kernel<bf16_t>, grid, block, 0, st, *a);
  else
    hipLaunchKernelGGL(hw_update_detect_kernel<float>, grid, block, 0, st, *a);
  return (int)hipGetLastError();
}
