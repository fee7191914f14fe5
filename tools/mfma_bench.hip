// Sustained v_mfma_f32_16x16x4_f32 rate vs independent accumulation chains per wave
// (C) and waves per SIMD (occupancy set by the workgroup size, one workgroup per CU).
//   hipcc --offload-arch=gfx950 -O3 tools/mfma_bench.hip -o tools/mfma_bench_bin
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float floatx4 __attribute__((ext_vector_type(4)));

template <int C>
__global__ void __launch_bounds__(1024) k(float* out, int iters, float a, float b) {
  floatx4 acc[C];
#pragma unroll
  for (int c = 0; c < C; ++c) acc[c] = floatx4{0.f, 0.f, 0.f, (float)c};
  const float x = a * threadIdx.x, y = b * threadIdx.x;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 16; ++u)
#pragma unroll
      for (int c = 0; c < C; ++c) acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(x, y, acc[c], 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < C; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int C>
void run(int threads, float* out) {
  const int blocks = 256, iters = 2000;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(k<C>, dim3(blocks), dim3(threads), 0, 0, out, 10, 1.f, 1.f);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k<C>, dim3(blocks), dim3(threads), 0, 0, out, iters, 1.f, 1.f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  const double mfmas = (double)blocks * (threads / 64) * iters * 16 * C;
  const double tflops = mfmas * 2048 / (ms * 1e-3) / 1e12;
  printf("chains %d  waves/SIMD %2d  %7.3f ms  %6.1f TFLOP/s  (%.0f%% of 157.3)\n", C, threads / 256, ms, tflops,
         100 * tflops / 157.3);
}

int main() {
  float* out;
  hipMalloc(&out, 256 * 1024 * 4);
  for (int t : {256, 512, 768, 1024}) {
    run<1>(t, out);
    run<2>(t, out);
    run<4>(t, out);
  }
  return 0;
}
