// K8: bivariate-normal scorer (two metrics per series pair).
//
// Semantics: foremast_amd/models/bivariate.py.  One 256-thread workgroup per
// pair: two ring-buffer rows (same geometry) are streamed once with shifted
// moment sums (jointly-valid points only), merged across the block, then
// each current point is scored by squared Mahalanobis distance; anomaly iff
// d^2 > thr^2 (thr in sigma units, lowered by the pairwise factor when the
// canary test rejected).
#include "common.h"
#include "detect.h"
#include "args.h"



extern __shared__ __attribute__((aligned(16))) char fm_biv_smem[];

template <typename TIN>
__global__ __launch_bounds__(256) void bivariate_kernel(const BivArgs a) {
  const int n = blockIdx.x, tid = threadIdx.x;
  float* red = (float*)fm_biv_smem;
  const TIN* rx = (const TIN*)a.hx + (long long)n * a.ld;
  const TIN* ry = (const TIN*)a.hy + (long long)n * a.ld;
  float sx = 0.f, sy = 0.f;
  bool has = false;
  float c = 0.f, ax = 0.f, ay = 0.f, axx = 0.f, axy = 0.f, ayy = 0.f;
  for (int i = tid; i < a.len; i += blockDim.x) {
    int p = a.head + i;
    if (p >= a.ring_len) p -= a.ring_len;
    const float x = to_f32<TIN>(rx[p]);
    const float y = to_f32<TIN>(ry[p]);
    if (x == x && y == y) {
      if (!has) { sx = x; sy = y; has = true; }
      const float dx = x - sx, dy = y - sy;
      c += 1.f; ax += dx; ay += dy; axx += dx * dx; axy += dx * dy; ayy += dy * dy;
    }
  }
  // per-thread centred moments
  const float mx_t = c > 0.f ? sx + ax / c : 0.f;
  const float my_t = c > 0.f ? sy + ay / c : 0.f;
  const float cxx_t = c > 0.f ? axx - ax * ax / c : 0.f;
  const float cxy_t = c > 0.f ? axy - ax * ay / c : 0.f;
  const float cyy_t = c > 0.f ? ayy - ay * ay / c : 0.f;
  const float N = blk_sum(c, red);
  const float mx = N > 0.f ? blk_sum(c * mx_t, red) / N : 0.f;
  const float my = N > 0.f ? blk_sum(c * my_t, red) / N : 0.f;
  const float dmx = mx_t - mx, dmy = my_t - my;
  const float Sxx = blk_sum(cxx_t + c * dmx * dmx, red);
  const float Sxy = blk_sum(cxy_t + c * dmx * dmy, red);
  const float Syy = blk_sum(cyy_t + c * dmy * dmy, red);
  const float inv = 1.f / fmaxf(N, 1.f);
  const float vxx = Sxx * inv + a.eps, vxy = Sxy * inv, vyy = Syy * inv + a.eps;
  float det = vxx * vyy - vxy * vxy;
  if (fabsf(det) < 1e-20f) det = 1e-20f;
  if (tid == 0) {
    a.mean[2 * (long long)n] = mx;
    a.mean[2 * (long long)n + 1] = my;
    a.cov[3 * (long long)n] = vxx - a.eps;
    a.cov[3 * (long long)n + 1] = vxy;
    a.cov[3 * (long long)n + 2] = vyy - a.eps;
  }
  float thr = a.threshold[n];
  if (a.differs && a.differs[n]) thr *= a.pw_scale;
  const float thr2 = thr * thr;
  const bool model_ok = N >= (float)a.min_valid;
  float cnt = 0.f, anyv = 0.f, sc = 0.f;
  for (int k = tid; k < a.C; k += blockDim.x) {
    const float x = a.cur[((long long)n * a.C + k) * 2];
    const float y = a.cur[((long long)n * a.C + k) * 2 + 1];
    float d2 = fm_nan();
    if (x == x && y == y) {
      const float dx = x - mx, dy = y - my;
      d2 = (vyy * dx * dx - 2.f * vxy * dx * dy + vxx * dy * dy) / det;
      anyv = 1.f;
      cnt += (model_ok && d2 > thr2) ? 1.f : 0.f;
      sc = fmaxf(sc, sqrtf(fmaxf(d2, 0.f)));
    }
    if (a.d2) a.d2[(long long)n * a.C + k] = d2;
  }
  cnt = blk_sum(cnt, red);
  anyv = blk_max(anyv, red);
  sc = blk_max(sc, red);
  if (tid == 0) {
    const int ic = (int)cnt;
    const int v = ic > 0 ? 1 : ((anyv > 0.f && model_ok) ? 0 : -1);
    a.count[n] = ic;
    a.verdict[n] = (signed char)v;
    a.score[n] = sc;
    if (a.app_id) {
      const int app = a.app_id[n];
      if (v == 1) atomicAdd(&a.app_stats[2 * app], 1);
      if (v >= 0) atomicAdd(&a.app_stats[2 * app + 1], 1);
    }
  }
}

extern "C" int fm_bivariate(const BivArgs* a, int bf16, hipStream_t st) {
  if (a->N <= 0) return 0;
  if (a->len < 0 || a->len > a->ring_len || a->head < 0 || a->head >= a->ring_len)
    return (int)hipErrorInvalidValue;
  if (bf16)
    hipLaunchKernelGGL(bivariate_kernel<bf16_t>, dim3(a->N), dim3(256), 256, st, *a);
  else
    hipLaunchKernelGGL(bivariate_kernel<float>, dim3(a->N), dim3(256), 256, st, *a);
  return (int)hipGetLastError();
}
