// K10 tick ingest: one launch per scoring tick for a shard of series.
//
// Streaming layout (foremast_amd/ingest/ringbuffer.py):
//   hist [N, R]      7-day history ring (bf16 or f32), one point per minute;
//   cur  [N, P*W]    current window, P pods x W slots (slot = tick mod W);
//   newv [N, P]      this tick's per-pod values (from the host ingest, H2D);
//   base [N, P*W]    optional baseline (old-pod) window, streamed the same way;
//   newb [N, P]
// Per series: the slot being overwritten holds the oldest points (age W); their
// pod-mean graduates into history at column hist_col, then the new per-pod
// values take the slot.  With a baseline stream (canary) it is the BASELINE
// pods' mean that graduates: the model history follows the stable version and
// the canary is never fitted into the model it is judged against.  Without one
// (continuous monitoring) the current pods' mean graduates.  One thread per
// series; everything the tick needs is touched once.  `zero` (optional, nzero int32
// words): per-tick counters the scoring kernels accumulate into (per-app health
// counters) are cleared here, in the tick's first launch, instead of by a fill.
#include "common.h"

template <typename TH>
__global__ __launch_bounds__(256) void tick_ingest_kernel(TH* __restrict__ hist, long long ld_h, int hist_col,
                                                          float* __restrict__ cur, long long ld_c, int P, int W,
                                                          int slot, const float* __restrict__ newv,
                                                          long long ld_n, int N, int graduate,
                                                          float* __restrict__ base, const float* __restrict__ newb,
                                                          const int* __restrict__ st, int* __restrict__ zero,
                                                          int nzero) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  for (int i = n; i < nzero; i += gridDim.x * blockDim.x) zero[i] = 0;
  if (n >= N) return;
  if (st) {  // per-tick ring state from device memory (HIP-graph replays): {hist_col, slot, graduate}
    hist_col = st[0];
    slot = st[1];
    graduate = st[2];
  }
  float s = 0.f, c = 0.f;
  if (base) {
    float* brow = base + (long long)n * ld_c;
    const float* nb = newb + (long long)n * ld_n;
    for (int p = 0; p < P; ++p) {
      const int col = p * W + slot;
      const float old = brow[col];
      if (old == old) { s += old; c += 1.f; }
      brow[col] = nb[p];
    }
  }
  float* row = cur + (long long)n * ld_c;
  const float* nv = newv + (long long)n * ld_n;
  for (int p = 0; p < P; ++p) {
    const int col = p * W + slot;
    const float old = row[col];
    if (!base && old == old) { s += old; c += 1.f; }
    row[col] = nv[p];
  }
  if (graduate) hist[(long long)n * ld_h + hist_col] = from_f32<TH>(c > 0.f ? s / c : fm_nan());
}

static int tick_ingest_launch(void* hist, long long ld_h, int hist_col, float* cur, long long ld_c, int P,
                              int W, int slot, const float* newv, long long ld_n, int N, int graduate,
                              float* base, const float* newb, int bf16, const int* state, int* zero, int nzero,
                              hipStream_t st) {
  if (N <= 0 && nzero <= 0) return 0;
  if (P <= 0 || W <= 0 || slot < 0 || slot >= W || hist_col < 0 || nzero < 0 || (nzero > 0 && !zero))
    return (int)hipErrorInvalidValue;
  const int work = N > nzero ? N : nzero;
  dim3 grid((work + 255) / 256), block(256);
  if (bf16)
    hipLaunchKernelGGL(tick_ingest_kernel<bf16_t>, grid, block, 0, st, (bf16_t*)hist, ld_h, hist_col, cur,
                       ld_c, P, W, slot, newv, ld_n, N, graduate, base, newb, state, zero, nzero);
  else
    hipLaunchKernelGGL(tick_ingest_kernel<float>, grid, block, 0, st, (float*)hist, ld_h, hist_col, cur, ld_c,
                       P, W, slot, newv, ld_n, N, graduate, base, newb, state, zero, nzero);
  return (int)hipGetLastError();
}

extern "C" int fm_tick_ingest(void* hist, long long ld_h, int hist_col, float* cur, long long ld_c, int P,
                              int W, int slot, const float* newv, long long ld_n, int N, int graduate,
                              float* base, const float* newb, int bf16, int* zero, int nzero, hipStream_t st) {
  return tick_ingest_launch(hist, ld_h, hist_col, cur, ld_c, P, W, slot, newv, ld_n, N, graduate, base, newb,
                            bf16, nullptr, zero, nzero, st);
}

// graph-replayable form: hist_col / slot / graduate are read from `state` (device int32
// {hist_col, slot, graduate}, valid ranges are the caller's contract: hist_col < R, slot < W)
extern "C" int fm_tick_ingest_dev(void* hist, long long ld_h, float* cur, long long ld_c, int P, int W,
                                  const float* newv, long long ld_n, int N, float* base, const float* newb,
                                  int bf16, const int* state, int* zero, int nzero, hipStream_t st) {
  if (!state) return (int)hipErrorInvalidValue;
  return tick_ingest_launch(hist, ld_h, 0, cur, ld_c, P, W, 0, newv, ld_n, N, 1, base, newb, bf16, state, zero,
                            nzero, st);
}

// Tick health table to the host without a DMA round trip: the table (a few
// KB of int32 app counters) is written straight into pinned host memory by a
// kernel queued behind the scoring kernels, with system-scope stores so the
// host sees it once the stream is synchronised.  A hipMemcpyAsync D2H here is
// a separate copy engine / blit operation with its own ~20 us queue turnaround
// per tick (profiles/canary_12k5_r2.md).
__global__ __launch_bounds__(256) void copy_to_host_kernel(int* __restrict__ dst, const int* __restrict__ src,
                                                            long long n) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    __hip_atomic_store(dst + i, src[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

extern "C" int fm_copy_to_host_i32(int* dst_host, const int* src, long long n, hipStream_t st) {
  if (n <= 0) return 0;
  if (!dst_host || !src) return (int)hipErrorInvalidValue;
  long long blocks = (n + 255) / 256;
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(copy_to_host_kernel, dim3((unsigned)blocks), dim3(256), 0, st, dst_host, src, n);
  return (int)hipGetLastError();
}

// Device-resident ring state for HIP-graph ticks: the first node of a replay
// advances the steady-state tick record {hist_col, slot, graduate, head} held
// in device memory (full ring: the graduating point overwrites the column at
// `head`, which then moves by one; the window slot cycles mod W) and copies
// the forecast horizons of the new slot from a device table, so a replay needs
// no host-to-device copy at all.
// Doorbell (optional): a tick graph enqueued before its input is released starts with this
// kernel spinning until the host's pinned counter `bell` reaches the replay's number
// (bell_dev[0] + 1, kept on the device so one captured graph serves every tick), so the
// tick starts a PCIe write after the host releases it instead of a graph launch after it.
// bell_dev[1] counts waits that gave up after `limit` wall-clock ticks (the tick then runs
// on whatever input it has; the host checks the count).
__global__ __launch_bounds__(256) void tick_advance_kernel(int* __restrict__ st, int R, int W,
                                                           const int* __restrict__ h_table, int nh,
                                                           int* __restrict__ h_buf, const int* bell,
                                                           int* __restrict__ bell_dev, long long limit) {
  if (bell) {
    if (threadIdx.x == 0) {
      const int want = bell_dev[0] + 1;
      const long long t0 = wall_clock64();
      while (__hip_atomic_load(bell, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < want) {
        if (wall_clock64() - t0 > limit) {
          bell_dev[1] += 1;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      bell_dev[0] = want;
    }
    __syncthreads();
  }
  const int head = st[3], slot = st[1];
  __syncthreads();  // every thread has the previous record before thread 0 rewrites it
  const int nslot = slot + 1 < W ? slot + 1 : 0;
  if (threadIdx.x == 0) {
    st[0] = head;                      // hist_col: the oldest column is overwritten
    st[1] = nslot;                     // this tick's window slot
    st[2] = 1;                         // graduate
    st[3] = head + 1 < R ? head + 1 : 0;
  }
  if (h_table) {
    const int hs = nslot + 1 < W ? nslot + 1 : 0;  // horizons after the tick (ticks + 1) mod W
    for (int i = threadIdx.x; i < nh; i += blockDim.x) h_buf[i] = h_table[(long long)hs * nh + i];
  }
}

extern "C" int fm_tick_advance(int* state, int R, int W, const int* h_table, int nh, int* h_buf, const int* bell,
                               int* bell_dev, long long limit, hipStream_t st) {
  if (!state || R <= 0 || W <= 0 || (h_table && (!h_buf || nh <= 0)) || (bell && (!bell_dev || limit <= 0)))
    return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(tick_advance_kernel, dim3(1), dim3(256), 0, st, state, R, W, h_table, nh, h_buf, bell, bell_dev,
                     limit);
  return (int)hipGetLastError();
}

// One-shot (canary / rollingUpdate) job windows (brain/rollout.py): row n holds
// one (job, metric) of a job that started at its own minute, laid out pod-major
// as P pods x Wc minutes of the job's current window (column c = minute c + 1
// after the job's start, so every row forecasts the same horizons).  A tick's
// decoded points arrive as src [S, k] (one row per (metric family, pod) the
// node watches, k consecutive minutes starting at the tick's first new minute);
// srcmap[n*P + p] is the src row of pod p of row n (-1: no such pod) and
// col0[n] the window column of the first minute for row n (negative / >= Wc:
// outside the job's window, dropped).  Missing points (NaN) never overwrite a
// value.  One thread per (row, pod, minute).
__global__ __launch_bounds__(256) void rollout_scatter_kernel(float* __restrict__ win, long long ld_w, int P, int Wc,
                                                              const float* __restrict__ src, long long ld_s, int k,
                                                              long long S, const int* __restrict__ srcmap,
                                                              const int* __restrict__ col0, int N) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long total = (long long)N * P * k;
  if (i >= total) return;
  const int j = (int)(i % k);
  const long long np = i / k;  // n * P + p
  const int n = (int)(np / P), p = (int)(np % P);
  const int c = col0[n] + j;
  if (c < 0 || c >= Wc) return;
  const long long sr = srcmap ? (long long)srcmap[np] : np;
  if (sr < 0 || sr >= S) return;
  const float v = src[sr * ld_s + j];
  if (v == v) win[(long long)n * ld_w + p * Wc + c] = v;
}

// The product tick's first kernel (brain/rollout.py): the same scatter with the window
// column computed in-kernel from the tick's first minute (a device scalar, so a captured
// HIP graph replays it unchanged) and the row's first-column minute, and the per-tick
// counters of the detection epilogue zeroed on the way (per-app counters, the K9 list
// count): one launch instead of four.
__global__ __launch_bounds__(256) void rollout_tick_scatter_kernel(float* __restrict__ win, long long ld_w, int P,
                                                                   int Wc, const float* __restrict__ src,
                                                                   long long ld_s, int k, long long S,
                                                                   const int* __restrict__ srcmap,
                                                                   const int* __restrict__ start_min,
                                                                   const int* __restrict__ tick, int N,
                                                                   int* __restrict__ zero_a, int n_a,
                                                                   int* __restrict__ zero_b, int n_b) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n_a) zero_a[i] = 0;
  if (i < n_b) zero_b[i] = 0;
  const long long total = (long long)N * P * k;
  if (i >= total) return;
  const int j = (int)(i % k);
  const long long np = i / k;  // n * P + p
  const int n = (int)(np / P), p = (int)(np % P);
  const int c = tick[0] - start_min[n] + j;
  if (c < 0 || c >= Wc) return;
  const long long sr = srcmap ? (long long)srcmap[np] : np;
  if (sr < 0 || sr >= S) return;
  const float v = src[sr * ld_s + j];
  if (v == v) win[(long long)n * ld_w + p * Wc + c] = v;
}

extern "C" int fm_rollout_tick_scatter(float* win, long long ld_w, int P, int Wc, const float* src, long long ld_s,
                                       int k, long long S, const int* srcmap, const int* start_min, const int* tick,
                                       int N, int* zero_a, int n_a, int* zero_b, int n_b, hipStream_t st) {
  if (P <= 0 || Wc <= 0 || k <= 0 || N < 0 || n_a < 0 || n_b < 0) return (int)hipErrorInvalidValue;
  long long total = (long long)N * P * k;
  if (total < n_a) total = n_a;
  if (total < n_b) total = n_b;
  if (total <= 0) return 0;
  hipLaunchKernelGGL(rollout_tick_scatter_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, win, ld_w,
                     P, Wc, src, ld_s, k, S, srcmap, start_min, tick, N, zero_a, n_a, zero_b, n_b);
  return (int)hipGetLastError();
}

extern "C" int fm_rollout_scatter(float* win, long long ld_w, int P, int Wc, const float* src, long long ld_s, int k,
                                  long long S, const int* srcmap, const int* col0, int N, hipStream_t st) {
  if (N <= 0 || k <= 0) return 0;
  if (!win || !src || !col0 || P <= 0 || Wc <= 0 || ld_w < (long long)P * Wc || ld_s < k || S < 0 ||
      (!srcmap && S < (long long)N * P))
    return (int)hipErrorInvalidValue;
  const long long total = (long long)N * P * k;
  hipLaunchKernelGGL(rollout_scatter_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, win, ld_w, P,
                     Wc, src, ld_s, k, S, srcmap, col0, N);
  return (int)hipGetLastError();
}
