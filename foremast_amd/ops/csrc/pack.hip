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
// fp8 (OCP e4m3) segments are block-scaled for v_mfma_scale_f32_32x32x64_f8f6f4 A
// fragments: codes index the logical [k-step][64 lanes][32 bytes]; the output is stored
// half-major, [k-step][16-byte half][64 lanes][16 bytes], so the kernel's 16-byte LDS
// reads of a fragment are lane-contiguous (conflict-free).  Measured on the MI355X
// (scripts/probe_mfma_scale.py): bytes 16 b .. 16 b + 15 of lanes r and r + 32 are one
// 32-value k block of row r, scaled by the E8M0 byte of lane r + 32 b.  A block's
// exponent e is the smallest integer with absmax <= 448 * 2^e (exact, from frexp); the
// codes are v * 2^-e in e4m3, and the scale bytes (e + 127) follow the codes lane-major
// (k-step s of lane l at n + l * (n / 2048) + s).  One pass: a block is a half wave.
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
  int _pad;
};

namespace {

__device__ __forceinline__ float fetch(const PackArgs& a, const PackSeg& s, int i) {
  const int c = s.code[i];
  if (c < 0) return 0.f;
  return a.src[(c >> 26) & 7][c & 0xffffff] * s.mul[(c >> 24) & 3];
}

// E8M0 exponent of a block with absolute maximum m (m = f 2^x, f in [0.5, 1); 448 = 0.875 2^9)
__device__ __forceinline__ int e8m0_exp(float m) {
  if (!(m > 0.f)) return 0;
  int x;
  const float f = frexpf(m, &x);
  const int e = x - 9 + (f > 0.875f ? 1 : 0);
  return e < -127 ? -127 : (e > 127 ? 127 : e);
}

__global__ __launch_bounds__(256) void pack_kernel(const PackArgs a) {
  const PackSeg& s = a.seg[blockIdx.y];
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (s.kind == 2) {  // block-scaled fp8 (n % 2048 == 0): half wave = block (k-step, row r, k block b)
    const int blk = i >> 5, u = i & 31;
    const int step = blk >> 6, r = blk & 31, b = (blk >> 5) & 1;
    const int lane = r + 32 * (u >> 4), j = 16 * b + (u & 15);
    const int e_idx = ((step << 6) + lane) * 32 + j;                       // logical [step][lane][32]
    const int o_idx = (step << 11) + (b << 10) + lane * 16 + (u & 15);     // stored half-major
    const float v = e_idx < s.n ? fetch(a, s, e_idx) : 0.f;
    float m = fabsf(v);
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, FM_WAVE));
    const int e = e8m0_exp(m);
    if (e_idx >= s.n) return;
    const int q = __builtin_amdgcn_cvt_pk_fp8_f32(ldexpf(v, -e), 0.f, 0, false);
    unsigned char* out = (unsigned char*)s.out;
    out[o_idx] = (unsigned char)(q & 0xff);
    if (u == 0) out[s.n + (r + 32 * b) * (s.n >> 11) + step] = (unsigned char)(e + 127);
    return;
  }
  if (i >= s.n) return;
  const float v = fetch(a, s, i);
  if (s.kind == 0)
    ((float*)s.out)[i] = v;
  else
    ((bf16_t*)s.out)[i] = f32_to_bf16(v);
}

}  // namespace

extern "C" int fm_pack(const PackArgs* a, hipStream_t st) {
  if (a->nseg <= 0 || a->nseg > 8) return (int)hipErrorInvalidValue;
  int maxn = 0;
  for (int s = 0; s < a->nseg; ++s) {
    if (a->seg[s].kind == 2 && a->seg[s].n % 2048) return (int)hipErrorInvalidValue;
    if (a->seg[s].n > maxn) maxn = a->seg[s].n;
  }
  if (maxn == 0) return 0;
  dim3 grid((unsigned)((maxn + 255) / 256), (unsigned)a->nseg), block(256);
  hipLaunchKernelGGL(pack_kernel, grid, block, 0, st, *a);
  return (int)hipGetLastError();
}

extern "C" long long fm_pack_args_size() { return (long long)sizeof(PackArgs); }
