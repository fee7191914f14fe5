// nc_adam.hip -- the Mapper's optimiser step over the grids and the colour decoder
// (torch.optim.Adam, src/Mapper.py:462-485 param groups, :625 optimizer.step()), and
// the lazy rule for sparse gradient rows (C5).
//
// k_adam_dense   thread = 4 consecutive elements (float4 when every operand is 16-B
//                aligned), grid-stride.  The arithmetic of torch.optim.Adam(fused=True)
//                (ATen fused_adam_utils.cuh adam_math, ORIGINAL mode, no amsgrad): the
//                moment updates are evaluated in double (beta1/beta2 are doubles) and
//                rounded to float, step size and denominator likewise, the parameter
//                update in float.  HBM-bound: 16 B read + 12 B written per element.
// k_adam_rows    thread = (row, channel) of a sparse gradient (nc_sparse_rows): the
//                rule of torch.optim.SparseAdam (torch/optim/_functional.py sparse_adam)
//                on the touched voxels only, all in float32 as its separate ATen ops
//                compute it.  Untouched voxels keep their parameter and moments.
#include "nc_internal.h"

namespace nc {

namespace {

// ATen's fused kernel is compiled with contraction on; on gfx950 its moment updates
// come out as fma(beta, moment, (1 - beta) * grad [* grad]) in double (measured against
// torch.optim.Adam(fused=True): the exact ties of 0.9 m + 0.1 g make the fused form
// observable).  Written out here; the library itself builds with -ffp-contract=off.
__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, double lr, double b1, double b2,
                                          double wd, double eps, float bc1, float bc2_sqrt) {
  if (wd != 0.0) g = (float)__builtin_fma((double)p, wd, (double)g);
  const double gd = g;
  m = (float)__builtin_fma(b1, (double)m, (1 - b1) * gd);
  v = (float)__builtin_fma(b2, (double)v, (1 - b2) * gd * gd);
  const float step_size = lr / bc1;
  const float denom = (double)(sqrtf(v) / bc2_sqrt) + eps;
  p -= step_size * m / denom;
}

}  // namespace

__global__ void __launch_bounds__(256) k_adam_dense(const nc_adam_args a, int vec) {
  // bias corrections from the step count as ATen computes them on the device (double),
  // handed to its adam_math as opmath (float) values
  const float bc1 = 1 - pow(a.beta1, a.step);
  const float bc2_sqrt = sqrt(1 - pow(a.beta2, a.step));
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t n4 = vec ? a.n / 4 : 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 p = reinterpret_cast<const float4*>(a.param)[i];
    const float4 g = reinterpret_cast<const float4*>(a.grad)[i];
    float4 m = reinterpret_cast<const float4*>(a.exp_avg)[i];
    float4 v = reinterpret_cast<const float4*>(a.exp_avg_sq)[i];
    adam_elem(p.x, g.x, m.x, v.x, a.lr, a.beta1, a.beta2, a.weight_decay, a.eps, bc1, bc2_sqrt);
    adam_elem(p.y, g.y, m.y, v.y, a.lr, a.beta1, a.beta2, a.weight_decay, a.eps, bc1, bc2_sqrt);
    adam_elem(p.z, g.z, m.z, v.z, a.lr, a.beta1, a.beta2, a.weight_decay, a.eps, bc1, bc2_sqrt);
    adam_elem(p.w, g.w, m.w, v.w, a.lr, a.beta1, a.beta2, a.weight_decay, a.eps, bc1, bc2_sqrt);
    reinterpret_cast<float4*>(a.param)[i] = p;
    reinterpret_cast<float4*>(a.exp_avg)[i] = m;
    reinterpret_cast<float4*>(a.exp_avg_sq)[i] = v;
  }
  for (int64_t i = n4 * 4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += stride) {
    float p = a.param[i], m = a.exp_avg[i], v = a.exp_avg_sq[i];
    adam_elem(p, a.grad[i], m, v, a.lr, a.beta1, a.beta2, a.weight_decay, a.eps, bc1, bc2_sqrt);
    a.param[i] = p;
    a.exp_avg[i] = m;
    a.exp_avg_sq[i] = v;
  }
}

// step_size = lr * sqrt(1 - beta2^step) / (1 - beta1^step), computed by the host in
// double like the reference's Python scalars; passed negated and rounded to float.
__global__ void __launch_bounds__(256) k_adam_rows(const nc_adam_args a, float neg_step_size, float omb1,
                                                   float omb2, float eps) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t r = t >> 5;
  const int c = (int)(t & 31);
  if (r >= a.row_capacity || r >= (int64_t)*a.row_count) return;
  const int64_t o = a.row_voxel[r] * a.voxel_stride + (int64_t)c * a.channel_stride;
  const float g = a.grad[r * 32 + c];
  const float m = a.exp_avg[o], v = a.exp_avg_sq[o];
  const float u1 = (g - m) * omb1;     // grad_values.sub(old_exp_avg_values).mul_(1 - beta1)
  const float u2 = (g * g - v) * omb2; // grad_values.pow(2).sub_(old_exp_avg_sq_values).mul_(1 - beta2)
  const float m1 = m + u1, v1 = v + u2;
  a.exp_avg[o] = m1;
  a.exp_avg_sq[o] = v1;
  const float denom = sqrtf(v1) + eps;
  a.param[o] = a.param[o] + neg_step_size * (m1 / denom);
}

// Many parameters per launch: block b belongs to the segment whose [blk_off[i],
// blk_off[i+1]) holds it; each segment is walked float4-wise (scalar when misaligned).
struct AdamSegs {
  nc_adam_segment seg[NC_ADAM_MAX_SEGMENTS];
  int32_t blk_off[NC_ADAM_MAX_SEGMENTS + 1];
  int32_t vec[NC_ADAM_MAX_SEGMENTS];
  int32_t n;
  double beta1, beta2, eps;
};

__global__ void __launch_bounds__(256) k_adam_multi(const AdamSegs S) {
  int i = 0;
  while (i + 1 < S.n && (int)blockIdx.x >= S.blk_off[i + 1]) ++i;
  const nc_adam_segment& g = S.seg[i];
  const double step = g.step_dev ? (double)*g.step_dev : g.step;
  const float bc1 = 1 - pow(S.beta1, step);
  const float bc2_sqrt = sqrt(1 - pow(S.beta2, step));
  const int64_t nb = S.blk_off[i + 1] - S.blk_off[i];
  const int64_t stride = nb * blockDim.x;
  const int64_t t0 = (int64_t)(blockIdx.x - S.blk_off[i]) * blockDim.x + threadIdx.x;
  const int64_t n4 = S.vec[i] ? g.n / 4 : 0;
  for (int64_t k = t0; k < n4; k += stride) {
    float4 p = reinterpret_cast<const float4*>(g.param)[k];
    const float4 gr = reinterpret_cast<const float4*>(g.grad)[k];
    float4 m = reinterpret_cast<const float4*>(g.exp_avg)[k];
    float4 v = reinterpret_cast<const float4*>(g.exp_avg_sq)[k];
    adam_elem(p.x, gr.x, m.x, v.x, g.lr, S.beta1, S.beta2, g.weight_decay, S.eps, bc1, bc2_sqrt);
    adam_elem(p.y, gr.y, m.y, v.y, g.lr, S.beta1, S.beta2, g.weight_decay, S.eps, bc1, bc2_sqrt);
    adam_elem(p.z, gr.z, m.z, v.z, g.lr, S.beta1, S.beta2, g.weight_decay, S.eps, bc1, bc2_sqrt);
    adam_elem(p.w, gr.w, m.w, v.w, g.lr, S.beta1, S.beta2, g.weight_decay, S.eps, bc1, bc2_sqrt);
    reinterpret_cast<float4*>(g.param)[k] = p;
    reinterpret_cast<float4*>(g.exp_avg)[k] = m;
    reinterpret_cast<float4*>(g.exp_avg_sq)[k] = v;
  }
  for (int64_t k = n4 * 4 + t0; k < g.n; k += stride) {
    float p = g.param[k], m = g.exp_avg[k], v = g.exp_avg_sq[k];
    adam_elem(p, g.grad[k], m, v, g.lr, S.beta1, S.beta2, g.weight_decay, S.eps, bc1, bc2_sqrt);
    g.param[k] = p;
    g.exp_avg[k] = m;
    g.exp_avg_sq[k] = v;
  }
}

constexpr int ADAM_COUNT_MAX = 256;
struct AdamCounts {
  float* step[ADAM_COUNT_MAX];
  int32_t n;
};
__global__ void k_adam_count(const AdamCounts C) {  // device step counts: += 1, one launch per call
  const int i = threadIdx.x;
  if (i < C.n) *C.step[i] += 1.f;
}

int launch_adam_multi(const nc_adam_args& a, const nc_adam_segment* segs, int n, hipStream_t s) {
  // blocks in proportion to each segment's float4 count, >= 1 each, ~4096 in total
  int64_t total = 0;
  for (int i = 0; i < n; ++i) total += (segs[i].n + 3) / 4;
  // device step counts first (capturable mode): every segment then reads its new count
  AdamCounts C{};
  for (int i = 0; i <= n; ++i) {
    if (C.n == ADAM_COUNT_MAX || (i == n && C.n > 0)) {
      hipLaunchKernelGGL(k_adam_count, dim3(1), dim3(ADAM_COUNT_MAX), 0, s, C);
      if (hipError_t e = hipGetLastError()) return (int)e;
      C.n = 0;
    }
    if (i < n && segs[i].step_dev) C.step[C.n++] = segs[i].step_dev;
  }
  for (int base = 0; base < n; base += NC_ADAM_MAX_SEGMENTS) {
    AdamSegs S{};
    S.n = std::min(n - base, NC_ADAM_MAX_SEGMENTS);
    S.beta1 = a.beta1;
    S.beta2 = a.beta2;
    S.eps = a.eps;
    int32_t off = 0;
    for (int i = 0; i < S.n; ++i) {
      const nc_adam_segment& g = segs[base + i];
      S.seg[i] = g;
      S.vec[i] = ((reinterpret_cast<uintptr_t>(g.param) | reinterpret_cast<uintptr_t>(g.grad) |
                   reinterpret_cast<uintptr_t>(g.exp_avg) | reinterpret_cast<uintptr_t>(g.exp_avg_sq)) & 15) == 0;
      const int64_t work = (g.n + 3) / 4;
      const int64_t want = std::min<int64_t>((work + 255) / 256, std::max<int64_t>(1, 4096 * work / std::max<int64_t>(total, 1)));
      S.blk_off[i] = off;
      off += (int32_t)std::max<int64_t>(want, 1);
    }
    S.blk_off[S.n] = off;
    hipLaunchKernelGGL(k_adam_multi, dim3((unsigned)off), dim3(256), 0, s, S);
    if (hipError_t e = hipGetLastError()) return (int)e;
  }
  return 0;
}

int launch_adam(const nc_adam_args& a, hipStream_t s) {
  if (a.mode == NC_ADAM_DENSE) {
    if (a.n == 0) return 0;
    const bool vec = ((reinterpret_cast<uintptr_t>(a.param) | reinterpret_cast<uintptr_t>(a.grad) |
                       reinterpret_cast<uintptr_t>(a.exp_avg) | reinterpret_cast<uintptr_t>(a.exp_avg_sq)) &
                      15) == 0;
    const int64_t work = vec ? (a.n + 3) / 4 : a.n;
    const int64_t blocks = std::min<int64_t>((work + 255) / 256, 256 * 16);
    hipLaunchKernelGGL(k_adam_dense, dim3((unsigned)blocks), dim3(256), 0, s, a, vec ? 1 : 0);
    return (int)hipGetLastError();
  }
  if (a.row_capacity == 0) return 0;
  const double bc1 = 1.0 - std::pow(a.beta1, a.step), bc2 = 1.0 - std::pow(a.beta2, a.step);
  const double step_size = a.lr * std::sqrt(bc2) / bc1;
  const int64_t blocks = (a.row_capacity * 32 + 255) / 256;
  hipLaunchKernelGGL(k_adam_rows, dim3((unsigned)blocks), dim3(256), 0, s, a, (float)-step_size,
                     (float)(1.0 - a.beta1), (float)(1.0 - a.beta2), (float)a.eps);
  return (int)hipGetLastError();
}

}  // namespace nc
