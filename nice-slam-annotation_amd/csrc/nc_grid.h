// nc_grid.h -- trilinear (grid_sample 3-D, border, align_corners) backward of a
// decoder's own grid lookup, restated from ATen's grid_sampler_3d_backward as the
// reference runs it through decoder.py:186 (and normalize_3d_coordinate,
// common.py:280-295): the coordinate gradient and the grid-gradient scatter of one
// wavefront's 16 points.  Called per tile by k_mlp_dx (nc_mlp.hip), right where the
// features' gradient is produced.
#pragma once
#include "nc_device.h"

namespace nc {

// coordinate gradient of one trilinear lookup (grid_sampler_3d_backward's
// gix/giy/giz): this lane's 8 channels; the caller sums the point's 4 lanes.
template <bool VEC>
__device__ __forceinline__ void grid_coord_grad(const nc_grid& G, const Corners& c, const float dc[8], int g,
                                                float gi[3]) {
  // branch-free in two batches of 4 corners (all 4 corners' loads in flight; an
  // out-of-bounds corner reads the in-bounds cell 0 and contributes 0), corner
  // order and association as the reference
  gi[0] = gi[1] = gi[2] = 0.f;
  const int64_t sC = G.stride[0];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    float v[4][8];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const float* base = G.data + c.off[4 * h + kk];
      if (VEC) {
        const float4 a = *reinterpret_cast<const float4*>(base + 4 * g);
        const float4 b = *reinterpret_cast<const float4*>(base + 16 + 4 * g);
        v[kk][0] = a.x; v[kk][1] = a.y; v[kk][2] = a.z; v[kk][3] = a.w;
        v[kk][4] = b.x; v[kk][5] = b.y; v[kk][6] = b.z; v[kk][7] = b.w;
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[kk][j] = base[(int64_t)feat_of(j, g) * sC];
      }
    }
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int k = 4 * h + kk;
      if (!((c.inb >> k) & 1u)) continue;  // out-of-bounds corner: no contribution
      const int xb = k & 1, yb = (k >> 1) & 1, zb = k >> 2;
      float dot = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) dot = dot + v[kk][j] * dc[j];
      gi[0] = gi[0] + (xb ? dot : -dot) * c.wy[yb] * c.wz[zb];
      gi[1] = gi[1] + (yb ? dot : -dot) * c.wx[xb] * c.wz[zb];
      gi[2] = gi[2] + (zb ? dot : -dot) * c.wx[xb] * c.wy[yb];
    }
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

}  // namespace nc
