// Host cost of a kernel launch on this stack (ROCm 7.2, MI355X): empty kernels with
// small and ~2 KB by-value arguments (k_mlp_fwd's MlpCtx is 1,872 B), enqueue time per
// launch without synchronisation.  hipcc --offload-arch=gfx950 -O2 tools/launch_cost.hip -o tools/launch_cost_bin
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

struct Big { char b[1872]; };
struct Mid { char b[1048]; };
__global__ void k_small(int x) { if (x == 12345) asm volatile(""); }
__global__ void k_mid(const Mid m) { if (m.b[0] == 123) asm volatile(""); }
__global__ void k_big(const Big m) { if (m.b[0] == 123) asm volatile(""); }

template <typename F>
double per_launch(F f, int n) {
  for (int i = 0; i < 100; ++i) f();
  (void)hipDeviceSynchronize();
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < n; ++i) f();
  auto t1 = std::chrono::steady_clock::now();
  (void)hipDeviceSynchronize();
  return std::chrono::duration<double, std::micro>(t1 - t0).count() / n;
}

int main() {
  hipStream_t s;
  (void)hipStreamCreate(&s);
  Big big{};
  Mid mid{};
  const int n = 20000;
  printf("small args, 1 block:     %.2f us/launch\n", per_launch([&] { hipLaunchKernelGGL(k_small, dim3(1), dim3(64), 0, s, 1); }, n));
  printf("1,048-B args, 250 blocks: %.2f us/launch\n", per_launch([&] { hipLaunchKernelGGL(k_mid, dim3(250), dim3(256), 0, s, mid); }, n));
  printf("1,872-B args, 256 blocks: %.2f us/launch\n", per_launch([&] { hipLaunchKernelGGL(k_big, dim3(256), dim3(512), 0, s, big); }, n));
  printf("1,872-B args + hipGetLastError: %.2f us/launch\n", per_launch([&] { hipLaunchKernelGGL(k_big, dim3(256), dim3(512), 0, s, big); (void)hipGetLastError(); }, n));
  int dev;
  printf("hipGetDevice:            %.3f us\n", per_launch([&] { (void)hipGetDevice(&dev); }, n));
  return 0;
}
