// Accuracy of sin/cos forms for the Fourier features (|x| up to ~1e3 rad):
// ocml sinf/cosf, __sinf/__cosf, and Cody-Waite reduction to [-pi,pi] followed by
// the hardware v_sin_f32 / v_cos_f32.  Errors vs double precision on the host.
//   hipcc --offload-arch=gfx950 -O3 tools/sin_accuracy.hip -o /tmp/sinacc && /tmp/sinacc
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

__device__ __forceinline__ float reduce_2pi(float x) {
  // x - k*2pi, k = rint(x / 2pi); 2pi split into three floats (Cody-Waite)
  const float k = __builtin_rintf(x * 0.15915494309189535f);
  float r = __builtin_fmaf(-k, 6.28125f, x);
  r = __builtin_fmaf(-k, 1.9353071795864769e-3f, r);
  r = __builtin_fmaf(-k, 1.2537033403800354e-11f, r);
  return r;
}
__device__ __forceinline__ float fast_sin(float x) {
  return __builtin_amdgcn_sinf(reduce_2pi(x) * 0.15915494309189535f);
}
__device__ __forceinline__ float fast_cos(float x) {
  return __builtin_amdgcn_cosf(reduce_2pi(x) * 0.15915494309189535f);
}

__global__ void k(const float* x, float* out, int n) {
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  float v = x[t];
  out[6 * t + 0] = sinf(v);
  out[6 * t + 1] = cosf(v);
  out[6 * t + 2] = __sinf(v);
  out[6 * t + 3] = __cosf(v);
  out[6 * t + 4] = fast_sin(v);
  out[6 * t + 5] = fast_cos(v);
}

int main() {
  const int n = 1 << 22;
  std::vector<float> x(n);
  std::mt19937 rng(1);
  std::uniform_real_distribution<float> u(-1000.f, 1000.f);
  for (int i = 0; i < n; ++i) x[i] = (i < n / 2) ? u(rng) : u(rng) * 1e-2f;
  float *dx, *dout;
  hipMalloc(&dx, n * 4);
  hipMalloc(&dout, n * 24);
  hipMemcpy(dx, x.data(), n * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3((n + 255) / 256), dim3(256), 0, 0, dx, dout, n);
  std::vector<float> o(6 * (size_t)n);
  hipMemcpy(o.data(), dout, n * 24, hipMemcpyDeviceToHost);
  const char* names[6] = {"sinf", "cosf", "__sinf", "__cosf", "cw+v_sin", "cw+v_cos"};
  for (int m = 0; m < 6; ++m) {
    double mx = 0, s2 = 0;
    for (int i = 0; i < n; ++i) {
      double ref = (m % 2 == 0) ? std::sin((double)x[i]) : std::cos((double)x[i]);
      double e = std::fabs((double)o[6 * (size_t)i + m] - ref);
      mx = e > mx ? e : mx;
      s2 += e * e;
    }
    printf("%-10s max abs err %.3e  rms %.3e\n", names[m], mx, std::sqrt(s2 / n));
  }
  return 0;
}
