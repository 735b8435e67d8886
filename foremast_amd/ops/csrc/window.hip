// K10 (device side) ring-buffer append and K1 window statistics
// (moving_average / moving_average_all) with the fused detection epilogue.
//
// Semantics: foremast_amd/ingest/ringbuffer.py and
// foremast_amd/models/moving_average.py.
#include "common.h"
#include "detect.h"
#include "args.h"

// ---------------------------------------------------------------------------------
// ring append: dst[n, (col0 + j) % R] = src[n, j]   (j < S)
// ---------------------------------------------------------------------------------
// col_dev (optional): a device int added to col0 (graph-captured ticks: the column moves
// every replay, the kernel argument cannot)
template <typename TOUT>
__global__ __launch_bounds__(256) void ring_append_kernel(TOUT* __restrict__ dst, long long ld_dst, int R,
                                                          int col0, const int* __restrict__ col_dev, int S,
                                                          const float* __restrict__ src, long long ld_src,
                                                          long long N) {
  if (col_dev) col0 = (col0 + col_dev[0]) % R;
  const long long total = N * (long long)S;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long n = i / S;
    const int j = (int)(i - n * S);
    int c = col0 + j;
    c %= R;
    dst[n * ld_dst + c] = from_f32<TOUT>(src[n * ld_src + j]);
  }
}

extern "C" int fm_ring_append_dev(void* dst, long long ld_dst, int R, int col0, const int* col_dev, int S,
                                  const float* src, long long ld_src, long long N, int bf16, hipStream_t st) {
  if (N <= 0 || S <= 0) return 0;
  if (R <= 0 || col0 < 0 || col0 >= R) return (int)hipErrorInvalidValue;
  long long total = N * (long long)S;
  long long blocks = (total + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (bf16)
    hipLaunchKernelGGL(ring_append_kernel<bf16_t>, dim3((unsigned)blocks), dim3(256), 0, st,
                       (bf16_t*)dst, ld_dst, R, col0, col_dev, S, src, ld_src, N);
  else
    hipLaunchKernelGGL(ring_append_kernel<float>, dim3((unsigned)blocks), dim3(256), 0, st,
                       (float*)dst, ld_dst, R, col0, col_dev, S, src, ld_src, N);
  return (int)hipGetLastError();
}

extern "C" int fm_ring_append(void* dst, long long ld_dst, int R, int col0, int S, const float* src,
                              long long ld_src, long long N, int bf16, hipStream_t st) {
  return fm_ring_append_dev(dst, ld_dst, R, col0, nullptr, S, src, ld_src, N, bf16, st);
}

// ---------------------------------------------------------------------------------
// window statistics + detection (one wave per series)
// ---------------------------------------------------------------------------------



// Accumulate shifted sums over physical range [p0, p1) of a row; vector body
// of 16-byte loads, scalar head/tail.
template <typename TIN, int UNR = 6>
__device__ __forceinline__ void acc_range(const TIN* row, int p0, int p1, float& shift, bool& has_shift,
                                          float& n, float& s1, float& s2, int tid, int nt) {
  constexpr int VEC = 16 / sizeof(TIN);
  auto add = [&](float v) {
    if (v == v) {
      if (!has_shift) { shift = v; has_shift = true; }
      const float d = v - shift;
      n += 1.f; s1 += d; s2 += d * d;
    }
  };
  int a0 = p0 + ((VEC - (p0 % VEC)) % VEC);
  if (a0 > p1) a0 = p1;
  for (int i = p0 + tid; i < a0; i += nt) add(to_f32<TIN>(row[i]));
  const int nvec = (p1 - a0) / VEC;
  // UNR 16-byte loads of a thread in flight at once (clamped index, no branch before the
  // loads), then the accumulation: one memory latency per UNR vectors instead of one each
  for (int v0 = tid; v0 < nvec; v0 += nt * UNR) {
    uint4 q[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) q[u] = *(const uint4*)(row + a0 + min(v0 + u * nt, nvec - 1) * VEC);
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      if (v0 + u * nt >= nvec) break;
      if (sizeof(TIN) == 2) {
        const unsigned w[4] = {q[u].x, q[u].y, q[u].z, q[u].w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          add(__uint_as_float(w[k] << 16));
          add(__uint_as_float(w[k] & 0xffff0000u));
        }
      } else {
        add(__uint_as_float(q[u].x)); add(__uint_as_float(q[u].y));
        add(__uint_as_float(q[u].z)); add(__uint_as_float(q[u].w));
      }
    }
  }
  for (int i = a0 + nvec * VEC + tid; i < p1; i += nt) add(to_f32<TIN>(row[i]));
}

// One wave per series (kSeriesPerWG per workgroup): the same statistics with wave
// reductions only, no workgroup barriers, and ~20 16-byte loads of a lane in flight in
// two batches.
constexpr int kWindowBlock = 256;
constexpr int kSeriesPerWG = kWindowBlock / FM_WAVE;

template <typename TIN>
__global__ __launch_bounds__(kWindowBlock) void window_stats_wave_kernel(const WindowArgs a) {
  const int n = blockIdx.x * kSeriesPerWG + wave_id();
  if (n >= a.N) return;  // wave-uniform
  const int lane = lane_id();
  const TIN* row = (const TIN*)a.hist + (long long)n * a.ld;
  float shift = 0.f, cnt = 0.f, s1 = 0.f, s2 = 0.f;
  bool has = false;
  const int p0 = a.head, p1 = a.head + a.len;
  if (p1 <= a.ring_len) {
    acc_range<TIN, 10>(row, p0, p1, shift, has, cnt, s1, s2, lane, FM_WAVE);
  } else {
    acc_range<TIN, 10>(row, p0, a.ring_len, shift, has, cnt, s1, s2, lane, FM_WAVE);
    acc_range<TIN, 10>(row, 0, p1 - a.ring_len, shift, has, cnt, s1, s2, lane, FM_WAVE);
  }
  // per-lane (n, mean, M2) -> Chan merge about the count-weighted mean of the lane means
  const float mean_t = cnt > 0.f ? shift + s1 / cnt : 0.f;
  const float m2_t = cnt > 0.f ? fmaxf(s2 - s1 * s1 / cnt, 0.f) : 0.f;
  const float N = wave_sum(cnt);
  const float sm = wave_sum(cnt * mean_t);
  const float ref = N > 0.f ? sm / N : 0.f;
  const float dm = mean_t - ref;
  const float M2 = wave_sum(m2_t + cnt * dm * dm);
  const float mean = ref;
  const float var = N > 0.f ? M2 / N : 0.f;
  const float sd = N > 0.f ? sqrtf(fmaxf(var, 0.f)) : fm_nan();
  if (lane == 0) {
    a.mean[n] = N > 0.f ? mean : fm_nan();
    a.stdv[n] = sd;
    a.count[n] = N;
  }
  detect_epilogue_wave(a.det, n, sd, N, [mean](int) { return mean; });
}

extern "C" int fm_window_stats(const WindowArgs* a, int bf16, hipStream_t st) {
  if (a->N <= 0) return 0;
  if (a->len < 0 || a->len > a->ring_len || a->head < 0 || a->head >= a->ring_len)
    return (int)hipErrorInvalidValue;
  if (bf16 && (a->ld % 8) != 0) return (int)hipErrorInvalidValue;
  if (!bf16 && (a->ld % 4) != 0) return (int)hipErrorInvalidValue;
  const dim3 wgrid((a->N + kSeriesPerWG - 1) / kSeriesPerWG);
  if (bf16)
    hipLaunchKernelGGL(window_stats_wave_kernel<bf16_t>, wgrid, dim3(kWindowBlock), 0, st, *a);
  else
    hipLaunchKernelGGL(window_stats_wave_kernel<float>, wgrid, dim3(kWindowBlock), 0, st, *a);
  return (int)hipGetLastError();
}
