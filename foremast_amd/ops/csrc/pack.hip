// Table-driven parameter gather / convert: one launch re-lays-out every
// weight matrix a training step produces into the fragment orders the LSTM
// kernels consume (and scatters the weight-gradient GEMM results back into
// the parameters' .grad buckets).  Replaces a chain of ~15 tiny torch
// index/convert/copy launches per tick, each of which cost more host launch
// time than GPU time.
//
// Each output element i of segment s is described by one int code:
//   code < 0            → 0
//   code = src << 26 | cls << 24 | off   → src[src][off] * mul[cls]
// The codes are built once on the host (foremast_amd/ops/pack.py) from the
// same index maps the PyTorch reference layouts use.
//
// fp8 (OCP e4m3) segments are scaled per segment by 448 / absmax: pass 0
// (which also writes every non-fp8 segment) reduces absmax with one atomic
// per wave, pass 1 quantises.  Consumers recompute the scale from the same
// absmax on the device (fp8_scale in lstm_common.h): no host round trip.
#include "common.h"

struct PackSeg {
  const int* code;
  void* out;
  int n;
  int kind;  // 0 f32, 1 bf16, 2 fp8 e4m3
  float mul[4];
};

struct PackArgs {
  const float* src[8];
  PackSeg seg[8];
  int nseg;
  int pass;
  float* absmax;  // [8] per segment (fp8 only)
};

namespace {

__device__ __forceinline__ float fetch(const PackArgs& a, const PackSeg& s, int i) {
  const int c = s.code[i];
  if (c < 0) return 0.f;
  return a.src[(c >> 26) & 7][c & 0xffffff] * s.mul[(c >> 24) & 3];
}

__global__ __launch_bounds__(256) void pack_kernel(const PackArgs a) {
  const PackSeg& s = a.seg[blockIdx.y];
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (a.pass == 0) {
    if (s.kind == 2) {
      const float v = i < s.n ? fabsf(fetch(a, s, i)) : 0.f;
      const float m = wave_max(v);
      if (lane_id() == 0 && m > 0.f)  // non-negative floats order like their bits
        atomicMax((unsigned*)&a.absmax[blockIdx.y], __float_as_uint(m));
      return;
    }
    if (i >= s.n) return;
    const float v = fetch(a, s, i);
    if (s.kind == 0)
      ((float*)s.out)[i] = v;
    else
      ((bf16_t*)s.out)[i] = f32_to_bf16(v);
    return;
  }
  if (s.kind != 2 || i >= s.n) return;
  const float m = a.absmax[blockIdx.y];
  const float inv = m > 0.f ? 448.f / m : 1.f;
  const int q = __builtin_amdgcn_cvt_pk_fp8_f32(fetch(a, s, i) * inv, 0.f, 0, false);
  ((unsigned char*)s.out)[i] = (unsigned char)(q & 0xff);
}

}  // namespace

extern "C" int fm_pack(const PackArgs* a, hipStream_t st) {
  if (a->nseg <= 0 || a->nseg > 8) return (int)hipErrorInvalidValue;
  int maxn = 0;
  bool fp8 = false;
  for (int s = 0; s < a->nseg; ++s) {
    if (a->seg[s].n > maxn) maxn = a->seg[s].n;
    fp8 |= a->seg[s].kind == 2;
  }
  if (maxn == 0) return 0;
  if (fp8) {
    if (!a->absmax) return (int)hipErrorInvalidValue;
    hipError_t e = hipMemsetAsync(a->absmax, 0, 8 * sizeof(float), st);
    if (e != hipSuccess) return (int)e;
  }
  dim3 grid((unsigned)((maxn + 255) / 256), (unsigned)a->nseg), block(256);
  PackArgs p = *a;
  p.pass = 0;
  hipLaunchKernelGGL(pack_kernel, grid, block, 0, st, p);
  if (fp8) {
    p.pass = 1;
    hipLaunchKernelGGL(pack_kernel, grid, block, 0, st, p);
  }
  return (int)hipGetLastError();
}

extern "C" long long fm_pack_args_size() { return (long long)sizeof(PackArgs); }
