// Probe of gfx950's v_permlane16_swap_b32 / v_permlane32_swap_b32 (the builtins return
// the pair {vdst, vsrc} after the swap): prints, per lane, the four results for
// vdst = vsrc = lane, to pin which halves an xor-16 / xor-32 exchange takes from each.
//   hipcc --offload-arch=gfx950 -O2 -o /tmp/permlane_probe tools/permlane_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void probe(int* out) {
  const unsigned v = threadIdx.x;
  const auto a = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  const auto b = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  out[threadIdx.x * 4 + 0] = (int)a[0];
  out[threadIdx.x * 4 + 1] = (int)a[1];
  out[threadIdx.x * 4 + 2] = (int)b[0];
  out[threadIdx.x * 4 + 3] = (int)b[1];
}

int main() {
  int* d = nullptr;
  if (hipMalloc(&d, 64 * 4 * sizeof(int)) != hipSuccess) return 1;
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
  int h[256];
  if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
  for (int l = 0; l < 64; ++l) printf("lane %2d: p16 {%2d %2d}  p32 {%2d %2d}\n", l, h[4 * l], h[4 * l + 1], h[4 * l + 2], h[4 * l + 3]);
  hipFree(d);
  return 0;
}
