// nc_grid.hip — trilinear (grid_sample 3-D, border, align_corners) backward of the
// decoders' own grid lookups: the grid-gradient scatter and the coordinate
// gradient, restated from ATen's grid_sampler_3d_backward as the reference runs
// it through decoder.py:186 (and normalize_3d_coordinate, common.py:280-295).
//
// Inputs come from k_mlp_bwd: d features per point (this decoder's 32 channels)
// and the Fourier part of the point gradient.  One wavefront owns 16 consecutive
// samples (usually of one ray).  Phase A (lane = point x channel group) computes
// the corners and the coordinate gradient; phase B (lane = channel, half-wave =
// point) issues the float atomics as whole 128-byte corner rows, summing runs of
// samples that fall in the same voxel cell on chip first.
#include "nc_device.h"
#include "nc_internal.h"

namespace nc {

// coordinate gradient of one trilinear lookup (grid_sampler_3d_backward's
// gix/giy/giz): this lane's 8 channels; the caller sums the point's 4 lanes.
template <bool VEC>
__device__ __forceinline__ void grid_coord_grad(const nc_grid& G, const Corners& c, const float dc[8], int g,
                                                float gi[3]) {
  gi[0] = gi[1] = gi[2] = 0.f;
  const int64_t sC = G.stride[0];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    if (!((c.inb >> k) & 1u)) continue;
    const int xb = k & 1, yb = (k >> 1) & 1, zb = k >> 2;
    const float* base = G.data + c.off[k];
    float v[8];
    if (VEC) {
      const float4 a = *reinterpret_cast<const float4*>(base + 4 * g);
      const float4 b = *reinterpret_cast<const float4*>(base + 16 + 4 * g);
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
      v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = base[(int64_t)feat_of(j, g) * sC];
    }
    float dot = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) dot = dot + v[j] * dc[j];
    gi[0] = gi[0] + (xb ? dot : -dot) * c.wy[yb] * c.wz[zb];
    gi[1] = gi[1] + (yb ? dot : -dot) * c.wx[xb] * c.wz[zb];
    gi[2] = gi[2] + (zb ? dot : -dot) * c.wx[xb] * c.wy[yb];
  }
}

// Grid-gradient scatter of one wave's 16 points (grid_sampler_3d_backward's
// gInput += w_k * gOut).  The point features' gradients (C layout) and corner
// tables go through a private LDS slice, then every float atomic instruction
// covers whole 128-byte corner rows (lane = channel, the two half-waves take
// different points), and consecutive samples of a ray that fall in the same
// voxel cell are summed on chip first (one atomic per corner per run).
constexpr int SCAT_FLOATS = 16 * 32 + 16 * 8 + 2 * 16 * 8 + 2 * 16 + 16 + 16;  // 976 (16-B multiple)

__device__ __forceinline__ void grid_scatter(const nc_grid& G, const Corners& c, const float dc[8], bool valid,
                                             float* reg, int i, int g, int lane) {
  float* D = reg;                                           // [16][32] d features
  float* Wt = reg + 512;                                    // [16][8] corner weights
  int64_t* OFF = reinterpret_cast<int64_t*>(reg + 640);     // [16][8] grad-corner offsets
  int64_t* KEY = reinterpret_cast<int64_t*>(reg + 896);     // [16] voxel-cell key (-1: none)
  int* INB = reinterpret_cast<int*>(reg + 928);             // [16] in-bounds corner mask
  *reinterpret_cast<float4*>(D + i * 32 + 4 * g) = float4{dc[0], dc[1], dc[2], dc[3]};
  *reinterpret_cast<float4*>(D + i * 32 + 16 + 4 * g) = float4{dc[4], dc[5], dc[6], dc[7]};
  // lane-group g writes corners 2g, 2g+1 of its point
  {
    // corners 2g, 2g+1: x bit = h, y bit = g&1, z bit = g>>1 (selects, not a runtime index)
    const int yb = g & 1, zb = g >> 1;
    const float wy = yb ? c.wy[1] : c.wy[0];
    const float wz = zb ? c.wz[1] : c.wz[0];
    const int64_t base = (c.z0 + zb) * G.grad_stride[1] + (c.y0 + yb) * G.grad_stride[2] + c.x0 * G.grad_stride[3];
    Wt[i * 8 + 2 * g] = (c.wx[0] * wy) * wz;
    Wt[i * 8 + 2 * g + 1] = (c.wx[1] * wy) * wz;
    OFF[i * 8 + 2 * g] = base;
    OFF[i * 8 + 2 * g + 1] = base + G.grad_stride[3];
  }
  if (g == 0) {
    // cell coordinates packed into the key (x | y << 21 | z << 42; grids < 2^21 per axis)
    KEY[i] = valid ? (c.x0 | (c.y0 << 21) | (c.z0 << 42)) : -1;
    INB[i] = valid ? (int)c.inb : 0;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int half = lane >> 5, ch = lane & 31;
  const int64_t chs = (int64_t)ch * G.grad_stride[0];
  float acc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] = 0.f;
  // Walk the half's 8 samples in order.  acc[k] holds corner k of the current cell.
  // Same cell: keep accumulating.  Next cell one step away along one axis: the 4
  // corners of the shared face carry over, the other 4 are flushed.  Otherwise all
  // 8 are flushed.  One atomic instruction = one 128-B corner row (lane = channel).
  int run = half * 8;
  int64_t cur = KEY[run];
  auto flush_k = [&](int pt, int k) {
    if ((INB[pt] >> k) & 1) atomicAdd(G.grad + OFF[pt * 8 + k] + chs, acc[k]);
  };
  for (int j = 0; j < 8; ++j) {
    const int pt = half * 8 + j;
    const int64_t kk = KEY[pt];
    if (kk != cur) {
      const int64_t d = kk - cur;  // exact for one-step moves (no borrow across fields)
      int axis = -1, dir = 0;
      if (cur >= 0 && kk >= 0) {
        if (d == 1) { axis = 0; dir = 1; }
        else if (d == -1) { axis = 0; dir = -1; }
        else if (d == (int64_t(1) << 21)) { axis = 1; dir = 1; }
        else if (d == -(int64_t(1) << 21)) { axis = 1; dir = -1; }
        else if (d == (int64_t(1) << 42)) { axis = 2; dir = 1; }
        else if (d == -(int64_t(1) << 42)) { axis = 2; dir = -1; }
      }
      if (axis < 0) {
#pragma unroll
        for (int k = 0; k < 8; ++k) { flush_k(run, k); acc[k] = 0.f; }
      } else {
        // corners with the axis bit == (dir > 0 ? 1 : 0) form the shared face: they
        // become the new cell's corners with the bit flipped
        const int bit = 1 << axis;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const bool leaving = ((k & bit) != 0) == (dir < 0);  // face not shared
          if (leaving) flush_k(run, k);
        }
        float nacc[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int src = k ^ bit;  // same corner in the old cell's numbering
          const bool from_old = ((k & bit) != 0) == (dir < 0);
          nacc[k] = from_old ? acc[src] : 0.f;
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] = nacc[k];
      }
      cur = kk;
    }
    const float dv = D[pt * 32 + ch];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = acc[k] + Wt[pt * 8 + k] * dv;
    run = pt;
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) flush_k(run, k);
}

__device__ __forceinline__ Job pick_job3(const Job (&jobs)[MAX_JOBS], unsigned y) {
  return y == 0 ? jobs[0] : (y == 1 ? jobs[1] : jobs[2]);
}

__global__ void __launch_bounds__(256) k_grid_bwd(const MlpCtx ctx) {
  __shared__ __attribute__((aligned(16))) float slices[4 * SCAT_FLOATS];
  const Job job = pick_job3(ctx.jobs, blockIdx.y);
  const int kind = job.kind;
  // constant-index selects (no dynamic indexing into the argument block)
  const nc_grid& G = kind == 0 ? ctx.grids[0] : kind == 1 ? ctx.grids[1] : kind == 2 ? ctx.grids[2] : ctx.grids[3];
  const nc_decoder_params& D = kind == 0 ? ctx.dec[0] : kind == 1 ? ctx.dec[1] : kind == 2 ? ctx.dec[2] : ctx.dec[3];
  const bool need_grid = job.need_grid && G.grad != nullptr;
  const bool need_coord = job.need_coord != 0;
  if (!need_grid && !need_coord) return;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
  float* slice = slices + wave * SCAT_FLOATS;
  const bool vec = grid_vec_ok(G);
  const int64_t ntiles = (ctx.P + 15) / 16;
  for (int64_t t = (int64_t)blockIdx.x * 4 + wave; t < ntiles; t += (int64_t)gridDim.x * 4) {
    const int64_t p = t * 16 + i;
    const bool valid = p < ctx.P;
    const float4 n = valid ? ctx.xyz[(int64_t)job.slot * ctx.P + p] : float4{-1.f, -1.f, -1.f, 0.f};
    const float xyz[3] = {n.x, n.y, n.z};
    Corners co;
    make_corners(G, xyz, co);
    float dc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (valid) {
      const float* src = ctx.dcbuf + ((int64_t)job.slot * ctx.P + p) * HID;
      const float4 a = *reinterpret_cast<const float4*>(src + 4 * g);
      const float4 b = *reinterpret_cast<const float4*>(src + 16 + 4 * g);
      dc[0] = a.x; dc[1] = a.y; dc[2] = a.z; dc[3] = a.w;
      dc[4] = b.x; dc[5] = b.y; dc[6] = b.z; dc[7] = b.w;
    }
    if (need_coord) {
      float gi[3];
      if (vec) grid_coord_grad<true>(G, co, dc, g, gi);
      else grid_coord_grad<false>(G, co, dc, g, gi);
      gi[0] = sum_groups(gi[0]) * co.gmx;
      gi[1] = sum_groups(gi[1]) * co.gmy;
      gi[2] = sum_groups(gi[2]) * co.gmz;
      if (valid && g == 0) {
        double* dst = ctx.dpts + ((int64_t)job.slot * ctx.P + p) * 3;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          // normalize_3d_coordinate backward ((g * 2) / (hi - lo)) + the Fourier part
          const double gg = ((double)gi[k] * 2.0) / (D.bound[k][1] - D.bound[k][0]);
          dst[k] = gg + dst[k];
        }
      }
    }
    if (need_grid) grid_scatter(G, co, dc, valid, slice, i, g, lane);
  }
}

// ---------------------------------------------------------------------------
// Forward trilinear lookups (MLP.sample_grid_feature, decoder.py:179-188, and the
// fine decoder's no-grad grid_middle lookup, :196-202) for every (point, job), as
// their own high-occupancy kernel so the decoder kernel reads contiguous features.
// Thread = (point, 4-channel chunk q): chunks 0-7 sample the job's own grid, 8-15
// (fine decoder) grid_middle -- unless the middle decoder of the same stage has the
// same bound, whose lookup is then written to both (MlpCtx::share_mid).  Corners and weights are make_corners (bit-identical
// to ATen's grid_sampler_3d); channels accumulate corner by corner without FMA.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_grid_gather(const MlpCtx ctx) {
  const unsigned y = blockIdx.y;
  const Job job = y == 0 ? ctx.jobs[0] : (y == 1 ? ctx.jobs[1] : ctx.jobs[2]);
  const int lg = (job.kind == K_FINE && !ctx.share_mid) ? 4 : 3;  // log2(chunks per point)
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t p = t >> lg;
  if (p >= ctx.P) return;
  const int q = (int)(t & ((1 << lg) - 1));
  const int gk = q < 8 ? job.kind : K_MID;
  // field-wise constant-index selects (a dynamic index into the kernel-argument
  // grid table would go through scratch)
  nc_grid G;
  G = gk == 0 ? ctx.grids[0] : gk == 1 ? ctx.grids[1] : gk == 2 ? ctx.grids[2] : ctx.grids[3];
  const float4 n = ctx.xyz[(int64_t)job.slot * ctx.P + p];
  const float xyz[3] = {n.x, n.y, n.z};
  Corners co;
  make_corners(G, xyz, co);
  const int c0 = 4 * (q & 7);
  const bool vec = grid_vec_ok(G);
  const int64_t sC = G.stride[0];
  float4 v[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const float* base = G.data + co.off[k] + (vec ? c0 : c0 * sC);
    if (vec) {
      v[k] = *reinterpret_cast<const float4*>(base);
    } else {
      v[k] = float4{base[0], base[sC], base[2 * sC], base[3 * sC]};
    }
  }
  float4 o = float4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const bool in = (co.inb >> k) & 1u;
    const float w = co.w[k];
    o.x = o.x + (in ? v[k].x * w : 0.f);
    o.y = o.y + (in ? v[k].y * w : 0.f);
    o.z = o.z + (in ? v[k].z * w : 0.f);
    o.w = o.w + (in ? v[k].w * w : 0.f);
  }
  *reinterpret_cast<float4*>(ctx.cfeat + job.c_off + p * job.c_stride + 4 * q) = o;
  if (ctx.share_mid && y == 1)  // the fine decoder's no-grad grid_middle lookup is this one
    *reinterpret_cast<float4*>(ctx.cfeat + ctx.jobs[0].c_off + p * ctx.jobs[0].c_stride + 32 + 4 * q) = o;
}

int launch_grid_gather(const MlpCtx& c, hipStream_t s) {
  const int64_t threads = c.P * 16;  // the widest job (fine: 16 chunks per point)
  hipLaunchKernelGGL(k_grid_gather, dim3((unsigned)((threads + 255) / 256), c.n_jobs), dim3(256), 0, s, c);
  return (int)hipGetLastError();
}

int launch_grid_bwd(const MlpCtx& c, hipStream_t s) {
  const int64_t ntiles = (c.P + 15) / 16;
  int64_t blocks = (ntiles + 3) / 4;
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(k_grid_bwd, dim3((unsigned)blocks, c.n_jobs), dim3(256), 0, s, c);
  return (int)hipGetLastError();
}

}  // namespace nc
