// mfma_rounding.hip -- how gfx950's MFMA rounds its accumulation (diagnostic tool, not product
// code).  D = C + sum_k a_k b_k for random operands with exactly representable products; the
// exact sum is formed in float64 on the host.  For each instruction the signed error e = D -
// exact is reported against the magnitude: a round-to-nearest accumulation gives
// mean(e * sign(exact)) / mean(|e|) near 0, a truncating one near -1 (every result pulled
// toward zero).  Compared with the float32 round-to-nearest of the exact sum.
//   hipcc --offload-arch=gfx950 -O3 -o tools/mfma_rounding_bin tools/mfma_rounding.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef _Float16 half8 __attribute__((ext_vector_type(8)));

// one wave per 16x16 block: D = C + A[16x32] B[32x16], f16 operands
__global__ void k_f16(const _Float16* A, const _Float16* B, const float* C, float* D) {
  const int l = threadIdx.x, i = l & 15, g = l >> 4;
  const int blk = blockIdx.x;
  A += blk * 16 * 32; B += blk * 32 * 16; C += blk * 256; D += blk * 256;
  half8 a, b;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    a[j] = A[i * 32 + 8 * g + j];
    b[j] = B[(8 * g + j) * 16 + i];
  }
  floatx4 c;
#pragma unroll
  for (int r = 0; r < 4; ++r) c[r] = C[(4 * g + r) * 16 + i];
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
#pragma unroll
  for (int r = 0; r < 4; ++r) D[(4 * g + r) * 16 + i] = c[r];
}

// D = C + A[16x4] B[4x16], f32 operands
__global__ void k_f32(const float* A, const float* B, const float* C, float* D) {
  const int l = threadIdx.x, i = l & 15, g = l >> 4;
  const int blk = blockIdx.x;
  A += blk * 16 * 4; B += blk * 4 * 16; C += blk * 256; D += blk * 256;
  floatx4 c;
#pragma unroll
  for (int r = 0; r < 4; ++r) c[r] = C[(4 * g + r) * 16 + i];
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(A[i * 4 + g], B[g * 16 + i], c, 0, 0, 0);
#pragma unroll
  for (int r = 0; r < 4; ++r) D[(4 * g + r) * 16 + i] = c[r];
}

static double urand() { return (rand() + 0.5) / ((double)RAND_MAX + 1.0); }

static void report(const char* name, const std::vector<float>& D, const std::vector<double>& X) {
  double se = 0, sa = 0, sr = 0, sra = 0;
  for (size_t n = 0; n < D.size(); ++n) {
    const double s = X[n] > 0 ? 1.0 : -1.0;
    const double e = (double)D[n] - X[n];
    const double er = (double)(float)X[n] - X[n];  // float32 round-to-nearest of the exact sum
    se += e * s; sa += fabs(e); sr += er * s; sra += fabs(er);
  }
  printf("%-34s mean(e sign)/mean|e| = %+.3f  mean|e|/mean|e_rne32| = %.2f   (rne32: %+.3f)\n", name, se / sa,
         sa / sra, sr / sra);
}

int main() {
  const int NB = 4096;
  srand(1);
  {  // f16 operands, f32 accumulator C of either sign
    std::vector<_Float16> A(NB * 512), B(NB * 512);
    std::vector<float> C(NB * 256), D(NB * 256);
    std::vector<double> X(NB * 256);
    for (auto& v : A) v = (_Float16)(urand() * 2 - 1);
    for (auto& v : B) v = (_Float16)(urand() * 2 - 1);
    for (auto& v : C) v = (float)((urand() * 2 - 1) * 4);
    for (int blk = 0; blk < NB; ++blk)
      for (int r = 0; r < 16; ++r)
        for (int c = 0; c < 16; ++c) {
          double s = C[blk * 256 + r * 16 + c];
          for (int k = 0; k < 32; ++k)
            s += (double)(float)A[blk * 512 + r * 32 + k] * (double)(float)B[blk * 512 + k * 16 + c];
          X[blk * 256 + r * 16 + c] = s;
        }
    _Float16 *dA, *dB; float *dC, *dD;
    hipMalloc(&dA, A.size() * 2); hipMalloc(&dB, B.size() * 2); hipMalloc(&dC, C.size() * 4); hipMalloc(&dD, D.size() * 4);
    hipMemcpy(dA, A.data(), A.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), B.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(dC, C.data(), C.size() * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_f16, dim3(NB), dim3(64), 0, 0, dA, dB, dC, dD);
    hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost);
    report("v_mfma_f32_16x16x32_f16", D, X);
    // C = 0: the products' sum alone
    std::vector<float> Z(C.size(), 0.f);
    hipMemcpy(dC, Z.data(), Z.size() * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_f16, dim3(NB), dim3(64), 0, 0, dA, dB, dC, dD);
    hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost);
    for (int blk = 0; blk < NB; ++blk)
      for (int n = 0; n < 256; ++n) X[blk * 256 + n] -= C[blk * 256 + n];
    report("v_mfma_f32_16x16x32_f16 (C = 0)", D, X);
    hipFree(dA); hipFree(dB); hipFree(dC); hipFree(dD);
  }
  {  // f32 operands
    std::vector<float> A(NB * 64), B(NB * 64), C(NB * 256), D(NB * 256);
    std::vector<double> X(NB * 256);
    for (auto& v : A) v = (float)(urand() * 2 - 1);
    for (auto& v : B) v = (float)(urand() * 2 - 1);
    for (auto& v : C) v = (float)((urand() * 2 - 1) * 2);
    for (int blk = 0; blk < NB; ++blk)
      for (int r = 0; r < 16; ++r)
        for (int c = 0; c < 16; ++c) {
          double s = C[blk * 256 + r * 16 + c];
          for (int k = 0; k < 4; ++k) s += (double)A[blk * 64 + r * 4 + k] * (double)B[blk * 64 + k * 16 + c];
          X[blk * 256 + r * 16 + c] = s;
        }
    float *dA, *dB, *dC, *dD;
    hipMalloc(&dA, A.size() * 4); hipMalloc(&dB, B.size() * 4); hipMalloc(&dC, C.size() * 4); hipMalloc(&dD, D.size() * 4);
    hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dC, C.data(), C.size() * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_f32, dim3(NB), dim3(64), 0, 0, dA, dB, dC, dD);
    hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost);
    report("v_mfma_f32_16x16x4_f32", D, X);
    hipFree(dA); hipFree(dB); hipFree(dC); hipFree(dD);
  }
  return 0;
}
