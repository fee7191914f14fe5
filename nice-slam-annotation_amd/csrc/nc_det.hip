// nc_det.hip -- NC_DETERMINISTIC grid-gradient scatter (SURVEY.md §8b "Determinism").
//
// The default backward scatters the trilinear grid gradient with float atomics inside
// k_mlp_dx (nc_grid.h), whose summation order varies run to run.  With
// NC_DETERMINISTIC, k_mlp_dx stores each point's feature gradient instead
// (MlpCtx::dfeat) and this file reduces them in a fixed order:
//   k_det_keys    entry (job, point, corner) -> key (job << vbits | voxel), weight
//   radix sort    rocprim's stable LSD radix sort of (key, entry id): the entries of
//                 one voxel end up adjacent, in ascending (point, corner) order
//   k_det_reduce  the first entry of each voxel run owns the voxel: it sums
//                 w * d feature over the run, channel per lane, in that order, and
//                 adds the sum to the gradient (unique owner: no atomics)
// The order is the reference's own: ATen's CPU grid_sampler_3d_backward walks points
// in order and adds each point's 8 corner contributions (gInp += gOut * w), and a
// voxel is a corner of a point at most once.
#include <rocprim/device/device_radix_sort.hpp>

#include "nc_device.h"
#include "nc_internal.h"

namespace nc {

__device__ __forceinline__ Job job_of(const MlpCtx& m, int j) {
  return j == 0 ? m.jobs[0] : (j == 1 ? m.jobs[1] : m.jobs[2]);
}
__device__ __forceinline__ nc_grid grid_of(const MlpCtx& m, int kind) {
  return kind == 0 ? m.grids[0] : kind == 1 ? m.grids[1] : kind == 2 ? m.grids[2] : m.grids[3];
}

__global__ void __launch_bounds__(256) k_det_keys(const MlpCtx m, DetBufs d) {
  const int j = blockIdx.y;
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= m.P) return;
  const Job job = job_of(m, j);
  const uint64_t invalid = (uint64_t(1) << (d.vbits + 2)) - 1;
  const int64_t e0 = ((int64_t)j * m.P + p) * 8;
  if (!job.need_grid) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      d.key[0][e0 + k] = invalid;
      d.val[0][e0 + k] = (uint32_t)(e0 + k);
      d.w[e0 + k] = 0.f;
    }
    return;
  }
  const nc_grid G = grid_of(m, job.kind);
  const float4 n = m.xyz[(int64_t)job.slot * m.P + p];
  const float xyz[3] = {n.x, n.y, n.z};
  Corners c;
  make_corners(G, xyz, c);
  const uint64_t H = (uint64_t)G.dims[1], W = (uint64_t)G.dims[2];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint64_t x = (uint64_t)(c.x0 + (k & 1)), y = (uint64_t)(c.y0 + ((k >> 1) & 1)),
                   z = (uint64_t)(c.z0 + (k >> 2));
    const bool in = (c.inb >> k) & 1u;
    d.key[0][e0 + k] = in ? (((uint64_t)j << d.vbits) | ((z * H + y) * W + x)) : invalid;
    d.val[0][e0 + k] = (uint32_t)(e0 + k);
    d.w[e0 + k] = c.w[k];
  }
}

// thread = (sorted entry e, channel ch); 8 entries per 256-thread block
__global__ void __launch_bounds__(256) k_det_reduce(const MlpCtx m, DetBufs d, int64_t n) {
  const int64_t e = (int64_t)blockIdx.x * 8 + (threadIdx.x >> 5);
  const int ch = threadIdx.x & 31;
  if (e >= n) return;
  const uint64_t* key = d.key[1];
  const uint64_t k0 = key[e];
  const uint64_t invalid = (uint64_t(1) << (d.vbits + 2)) - 1;
  if (k0 == invalid || (e > 0 && key[e - 1] == k0)) return;
  float acc = 0.f;
  for (int64_t q = e; q < n && key[q] == k0; ++q) {
    const uint32_t ent = d.val[1][q];
    acc = acc + m.dfeat[(int64_t)(ent >> 3) * 32 + ch] * d.w[ent];
  }
  const int j = (int)(k0 >> d.vbits);
  const uint64_t v = k0 & ((uint64_t(1) << d.vbits) - 1);
  const nc_grid G = grid_of(m, job_of(m, j).kind);
  const uint64_t H = (uint64_t)G.dims[1], W = (uint64_t)G.dims[2];
  const int64_t x = (int64_t)(v % W), y = (int64_t)((v / W) % H), z = (int64_t)(v / (W * H));
  if (G.grad_rows) {  // sparse gradient rows (claimed by the forward)
    const int r = G.grad_rows[v];
    if (r >= 0) G.grad[(int64_t)r * 32 + ch] += acc;
    return;
  }
  float* dst = G.grad + z * G.grad_stride[1] + y * G.grad_stride[2] + x * G.grad_stride[3] +
               (int64_t)ch * G.grad_stride[0];
  *dst = *dst + acc;
}

size_t det_sort_temp_bytes(int64_t n_entries, int end_bit) {
  size_t bytes = 0;
  if (rocprim::radix_sort_pairs(nullptr, bytes, (uint64_t*)nullptr, (uint64_t*)nullptr, (uint32_t*)nullptr,
                                (uint32_t*)nullptr, (size_t)n_entries, 0, (unsigned)end_bit) != hipSuccess)
    return 0;
  return bytes ? bytes : 1;
}

int launch_det_scatter(const MlpCtx& m, const DetBufs& d, hipStream_t s) {
  const int64_t n = (int64_t)m.n_jobs * m.P * 8;
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_det_keys, dim3((unsigned)((m.P + 255) / 256), m.n_jobs), dim3(256), 0, s, m, d);
  if (hipError_t e = hipGetLastError()) return (int)e;
  size_t bytes = d.temp_bytes;
  if (hipError_t e = rocprim::radix_sort_pairs(d.temp, bytes, d.key[0], d.key[1], d.val[0], d.val[1], (size_t)n, 0,
                                               (unsigned)(d.vbits + 2), s))
    return (int)e;
  hipLaunchKernelGGL(k_det_reduce, dim3((unsigned)((n + 7) / 8)), dim3(256), 0, s, m, d, n);
  return (int)hipGetLastError();
}

}  // namespace nc
