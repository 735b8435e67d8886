// Packed vs scalar FP32 FMA throughput on one MI355X (gfx950): 8 independent chains per
// thread, 4096 iterations, 1024 workgroups x 256 threads.  Prints TFLOP/s of each form.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float v2f __attribute__((ext_vector_type(2)));
constexpr int ITERS = 4096;

__global__ __launch_bounds__(256) void k_packed(float* out, float a, float b) {
  v2f acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = (v2f){(float)threadIdx.x + i, (float)i};
  const v2f va = (v2f){a, a}, vb = (v2f){b, b};
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = acc[i] * va + vb;  // v_pk_fma_f32
  }
  v2f s = acc[0];
  for (int i = 1; i < 8; ++i) s += acc[i];
  out[blockIdx.x * 256 + threadIdx.x] = s.x + s.y;
}

__global__ __launch_bounds__(256) void k_scalar(float* out, float a, float b) {
  float acc[16];
  for (int i = 0; i < 16; ++i) acc[i] = (float)threadIdx.x + i;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      float x = acc[i];
      asm volatile("v_fma_f32 %0, %1, %2, %3" : "=v"(x) : "v"(x), "v"(a), "v"(b));  // one lane-op each
      acc[i] = x;
    }
  }
  float s = 0.f;
  for (int i = 0; i < 16; ++i) s += acc[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_packed_asm(float* out, float a, float b) {
  v2f acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = (v2f){(float)threadIdx.x + i, (float)i};
  const v2f va = (v2f){a, a}, vb = (v2f){b, b};
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      v2f x = acc[i];
      asm volatile("v_pk_fma_f32 %0, %1, %2, %3" : "=v"(x) : "v"(x), "v"(va), "v"(vb));
      acc[i] = x;
    }
  }
  v2f s = acc[0];
  for (int i = 1; i < 8; ++i) s += acc[i];
  out[blockIdx.x * 256 + threadIdx.x] = s.x + s.y;
}

int main() {
  const int blocks = 1024 * 4;
  float* out;
  hipMalloc(&out, blocks * 256 * sizeof(float));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const double flops = 2.0 * 16 * ITERS * (double)blocks * 256;  // 16 FMA lanes per thread per iteration
  for (int rep = 0; rep < 3; ++rep) {
    for (int which = 0; which < 3; ++which) {
      hipEventRecord(e0);
      if (which == 0) hipLaunchKernelGGL(k_packed, dim3(blocks), dim3(256), 0, 0, out, 0.999f, 0.001f);
      if (which == 1) hipLaunchKernelGGL(k_scalar, dim3(blocks), dim3(256), 0, 0, out, 0.999f, 0.001f);
      if (which == 2) hipLaunchKernelGGL(k_packed_asm, dim3(blocks), dim3(256), 0, 0, out, 0.999f, 0.001f);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0.f;
      hipEventElapsedTime(&ms, e0, e1);
      printf("%s rep %d: %.3f ms  %.1f TFLOP/s\n", which == 0 ? "packed (compiler)" : which == 1 ? "scalar v_fma_f32" : "packed v_pk_fma_f32 asm", rep, ms, flops / ms / 1e9);
    }
  }
  hipFree(out);
  return 0;
}
