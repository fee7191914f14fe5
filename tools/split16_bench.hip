// split16_bench.hip -- numerics and rate of the "3 x f16" split MFMA product on gfx950
// against the exact-f32 v_mfma_f32_16x16x4_f32 chain (diagnostic tool, not product code).
//
// x = hi + lo / 2^11 with hi = f16(x), lo = f16((x - hi) * 2^11); the product
// sum_k a_k b_k is formed as  acc_hh + (acc_hl + acc_lh) / 2^11  from three
// v_mfma_f32_16x16x32_f16 (K = 32 per instruction), two accumulators.
//   hipcc --offload-arch=gfx950 -O3 -o tools/split16_bin tools/split16_bench.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef _Float16 half8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ void split8(const float* x, half8& hi, half8& lo) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const _Float16 h = (_Float16)x[j];
    hi[j] = h;
    lo[j] = (_Float16)((x[j] - (float)h) * 2048.f);
  }
}

// One wave: D[16x16] = A[16xK] * B[Kx16], K multiple of 32.  A row-major [16][K], B [K][16].
__global__ void k_split(const float* A, const float* B, float* D, int K, int reps) {
  const int l = threadIdx.x, i = l & 15, g = l >> 4;
  floatx4 hh = {0, 0, 0, 0}, mx = {0, 0, 0, 0};
  for (int rep = 0; rep < reps; ++rep) {
    for (int k0 = 0; k0 < K; k0 += 32) {
      float a[8], b[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        a[j] = A[i * K + k0 + 8 * g + j];
        b[j] = B[(k0 + 8 * g + j) * 16 + i];
      }
      half8 ah, al, bh, bl;
      split8(a, ah, al);
      split8(b, bh, bl);
      hh = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, hh, 0, 0, 0);
      mx = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, mx, 0, 0, 0);
      mx = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, mx, 0, 0, 0);
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) D[(4 * g + r) * 16 + i] = hh[r] + mx[r] * (1.f / 2048.f);
}

__global__ void k_f32(const float* A, const float* B, float* D, int K) {
  const int l = threadIdx.x, i = l & 15, g = l >> 4;
  floatx4 acc = {0, 0, 0, 0};
  for (int k0 = 0; k0 < K; k0 += 4)
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(A[i * K + k0 + g], B[(k0 + g) * 16 + i], acc, 0, 0, 0);
#pragma unroll
  for (int r = 0; r < 4; ++r) D[(4 * g + r) * 16 + i] = acc[r];
}

// throughput: operands in registers, 4 independent 3-MFMA groups per k-step
__global__ void k_rate_split(float* out, int iters) {
  half8 a, b;
#pragma unroll
  for (int j = 0; j < 8; ++j) { a[j] = (_Float16)(0.001f * (threadIdx.x + j)); b[j] = (_Float16)(0.002f * j); }
  floatx4 c[8] = {};
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int t = 0; t < 8; ++t) c[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c[t], 0, 0, 0);
  float s = 0;
#pragma unroll
  for (int t = 0; t < 8; ++t) s += c[t][0] + c[t][1] + c[t][2] + c[t][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_rate_f32(float* out, int iters) {
  float a = 0.001f * threadIdx.x, b = 0.002f;
  floatx4 c[8] = {};
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int t = 0; t < 8; ++t) c[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c[t], 0, 0, 0);
  float s = 0;
#pragma unroll
  for (int t = 0; t < 8; ++t) s += c[t][0] + c[t][1] + c[t][2] + c[t][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

static double urand(unsigned& s) { s = s * 1664525u + 1013904223u; return (s >> 8) * (1.0 / 16777216.0); }

int main() {
  const int Ks[] = {32, 128, 640};
  const double scales[] = {1.0, 1e-3, 1e-5, 300.0};
  for (int K : Ks)
    for (double sc : scales) {
      std::vector<float> A(16 * K), B(K * 16), D1(256), D2(256);
      unsigned s = 12345u + K;
      for (auto& v : A) v = (float)((urand(s) * 2 - 1) * sc);
      for (auto& v : B) v = (float)((urand(s) * 2 - 1) * 0.3);
      float *dA, *dB, *dD;
      hipMalloc(&dA, A.size() * 4); hipMalloc(&dB, B.size() * 4); hipMalloc(&dD, 256 * 4);
      hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
      hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice);
      k_split<<<1, 64>>>(dA, dB, dD, K, 1);
      hipMemcpy(D1.data(), dD, 1024, hipMemcpyDeviceToHost);
      k_f32<<<1, 64>>>(dA, dB, dD, K);
      hipMemcpy(D2.data(), dD, 1024, hipMemcpyDeviceToHost);
      double e1 = 0, e2 = 0, mag = 0;
      for (int r = 0; r < 16; ++r)
        for (int c = 0; c < 16; ++c) {
          double ref = 0, ab = 0;
          for (int k = 0; k < K; ++k) { ref += (double)A[r * K + k] * B[k * 16 + c]; ab += std::fabs((double)A[r * K + k] * B[k * 16 + c]); }
          e1 = std::fmax(e1, std::fabs(D1[r * 16 + c] - ref) / ab);
          e2 = std::fmax(e2, std::fabs(D2[r * 16 + c] - ref) / ab);
          mag = std::fmax(mag, ab);
        }
      printf("K=%4d |a|~%-7g  max err / sum|ab|: split16 %.3e   f32 %.3e\n", K, sc, e1, e2);
      hipFree(dA); hipFree(dB); hipFree(dD);
    }
  float* o;
  hipMalloc(&o, 256 * 4 * 256 * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  const int iters = 20000;
  for (int w = 0; w < 2; ++w) {
    hipEventRecord(e0);
    k_rate_split<<<1024, 256>>>(o, iters);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    double fl = 1024.0 * 4 * iters * 8 * 16 * 16 * 32 * 2;
    printf("f16 16x16x32: %.1f TFLOP/s\n", fl / ms / 1e9);
    hipEventRecord(e0);
    k_rate_f32<<<1024, 256>>>(o, iters);
    hipEventRecord(e1); hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    fl = 1024.0 * 4 * iters * 8 * 16 * 16 * 4 * 2;
    printf("f32 16x16x4 : %.1f TFLOP/s\n", fl / ms / 1e9);
  }
  return 0;
}
