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
      // out-of-bounds corners read cell 0
      const int k = 4 * h + kk;
      // VEC: out-of-bounds corners read the zero row (their dot is 0); else cell 0, skipped below
      const float* base = VEC ? corner_row(G, c, k) : G.data + corner_off(G, c, k);
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
    __builtin_amdgcn_sched_barrier(0);  // the batch's loads all issue before the first is consumed
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int k = 4 * h + kk;
      if (!VEC && !((c.inb >> k) & 1u)) continue;  // out-of-bounds corner: no contribution
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
// tables go through a private LDS slice.  Lane = (x side of the corner, channel):
// both half-waves walk the same 16 samples in lockstep, each holding the 4 corners
// of its x side, so every control decision is wave-uniform and every float atomic
// instruction covers two whole, adjacent 128-B corner rows (x0 and x0+1 of one
// (y, z): contiguous in channels-last).  Consecutive samples of a ray in the same
// voxel cell are summed on chip (one add per corner per run); a step to a
// face-adjacent cell carries the shared face over.  Sparse gradient rows
// (G.grad_rows): a corner's destination is its voxel's row instead of its voxel.
// Slice layout (floats), padded so the per-lane writes of the 16 points spread over
// the LDS banks: D [16][36] (row pad 4), Wt [x side][point][(y, z)] (one float4 per
// point and side in the walk), OFF transposed [corner][17].
constexpr int SCAT_DLD = 36, SCAT_KLD = 17;
constexpr int SCAT_WT = 16 * SCAT_DLD;             // 576
constexpr int SCAT_OFF = SCAT_WT + 8 * SCAT_KLD;   // 712 (8-B aligned)
constexpr int SCAT_KEY = SCAT_OFF + 2 * 8 * SCAT_KLD;  // 984
constexpr int SCAT_INB = SCAT_KEY + 2 * 16;        // 1016
constexpr int SCAT_FLOATS = SCAT_INB + 16;         // 1032 (16-B multiple)
static_assert(SCAT_FLOATS % 4 == 0 && SCAT_OFF % 2 == 0 && SCAT_KEY % 2 == 0, "scatter slice alignment");

// (1) staging: every lane of the wave that owns the 16 points writes its share
__device__ __forceinline__ void grid_scatter_stage(const nc_grid& G, const Corners& c, const float dc[8], bool valid,
                                                   float* reg, int i, int g) {
  float* D = reg;                                              // [16][36] d features
  float* Wt = reg + SCAT_WT;                                   // [2 x side][16][4 (y, z)] corner weights
  int64_t* OFF = reinterpret_cast<int64_t*>(reg + SCAT_OFF);   // [8][17] grad-corner offsets
  int64_t* KEY = reinterpret_cast<int64_t*>(reg + SCAT_KEY);   // [16] voxel-cell key (-1: none)
  int* INB = reinterpret_cast<int*>(reg + SCAT_INB);           // [16] in-bounds corner mask
  *reinterpret_cast<float4*>(D + i * SCAT_DLD + 4 * g) = float4{dc[0], dc[1], dc[2], dc[3]};
  *reinterpret_cast<float4*>(D + i * SCAT_DLD + 16 + 4 * g) = float4{dc[4], dc[5], dc[6], dc[7]};
  {
    const int yb = g & 1, zb = g >> 1;
    const float wy = yb ? c.wy[1] : c.wy[0];
    const float wz = zb ? c.wz[1] : c.wz[0];
    Wt[4 * i + g] = (c.wx[0] * wy) * wz;  // corner k = 2 g: x side 0, (y, z) = g
    Wt[64 + 4 * i + g] = (c.wx[1] * wy) * wz;
    if (G.grad_rows) {  // sparse gradient rows: the rows the forward claimed (-1: none, skipped)
      const int64_t v = ((int64_t)(c.z0 + zb) * G.dims[1] + (c.y0 + yb)) * G.dims[2] + c.x0;
      const int k0 = 2 * g, k1 = 2 * g + 1;
      const int r0 = ((c.inb >> k0) & 1u) ? G.grad_rows[v] : -1;
      const int r1 = ((c.inb >> k1) & 1u) ? G.grad_rows[v + 1] : -1;
      OFF[k0 * SCAT_KLD + i] = r0 < 0 ? -1 : (int64_t)r0 * 32;
      OFF[k1 * SCAT_KLD + i] = r1 < 0 ? -1 : (int64_t)r1 * 32;
    } else {
      const int64_t base = voxel_off(G.grad_stride, c.x0, c.y0 + yb, c.z0 + zb);
      OFF[(2 * g) * SCAT_KLD + i] = base;
      OFF[(2 * g + 1) * SCAT_KLD + i] = base + stride32(G.grad_stride[3]);
    }
  }
  if (g == 0) {
    KEY[i] = valid ? ((int64_t)c.x0 | ((int64_t)c.y0 << 21) | ((int64_t)c.z0 << 42)) : -1;
    INB[i] = valid ? (int)c.inb : 0;
  }
}

// (2) the walk over the staged 16 samples and the float atomics, by any one wave
// (the staging wave itself, or a scatter wave of the workgroup: k_mlp_dx)
__device__ __forceinline__ void grid_scatter_flush(const nc_grid& G, const float* reg, int lane) {
  const float* D = reg;
  const float* Wt = reg + SCAT_WT;
  const int64_t* OFF = reinterpret_cast<const int64_t*>(reg + SCAT_OFF);
  const int64_t* KEY = reinterpret_cast<const int64_t*>(reg + SCAT_KEY);
  const int* INB = reinterpret_cast<const int*>(reg + SCAT_INB);
  const int half = lane >> 5, ch = lane & 31;
  const int64_t chs = G.grad_rows ? (int64_t)ch : (int64_t)ch * stride32(G.grad_stride[0]);
  // the cell keys and in-bounds masks are per point, the same in every lane: read them
  // into scalar registers, so the walk's run / face-shift decisions are scalar branches
  auto key_at = [&](int pt) -> int64_t {
    const uint64_t v = (uint64_t)KEY[pt];
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return (int64_t)(((uint64_t)hi << 32) | lo);
  };
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  // up to four corner rows of point pt: every destination offset is read before the first
  // atomic is issued (one LDS wait per group, not one per atomic)
  auto flush_n = [&](int pt, int n, const int* k, const float* v) {
    int64_t o[4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
      if (a < n) o[a] = OFF[k[a] * SCAT_KLD + pt];
    const unsigned inb = __builtin_amdgcn_readfirstlane(INB[pt]);
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      if (a >= n) break;
      if (((inb >> k[a]) & 1u) && o[a] >= 0) atomicAdd(G.grad + o[a] + chs, v[a]);
    }
  };
  int run = 0;
  int64_t cur = key_at(0);
#ifdef NC_SCAT_UNROLL
#pragma unroll NC_SCAT_UNROLL
#endif
  for (int pt = 0; pt < 16; ++pt) {
    const int64_t kk = key_at(pt);  // wave-uniform
    // this point's d feature and corner weights, read before a run flush can wait on LDS
    const float dv = D[pt * SCAT_DLD + ch];
    const float4 w = *reinterpret_cast<const float4*>(Wt + 64 * half + 4 * pt);  // one read: this side's 4 corners
    if (kk != cur) {
      const int64_t d = kk - cur;
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
        const int k[4] = {half, half | 2, half | 4, half | 6};
        flush_n(run, 4, k, acc);
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[q] = 0.f;
      } else if (axis == 0) {
        const int L = dir > 0 ? 0 : 1;
        float mv[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) mv[q] = __shfl_xor(acc[q], 32);
        const bool onL = half == L;
        const int k[2] = {L | ((onL ? 0 : 2) << 1), L | ((onL ? 1 : 3) << 1)};
        const float v[2] = {onL ? acc[0] : mv[2], onL ? acc[1] : mv[3]};
        flush_n(run, 2, k, v);
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[q] = onL ? mv[q] : 0.f;
      } else {
        // the two (y, z) corners on the far side of the shared face leave (the axis and
        // direction are scalar: which two q is the same in every lane)
        const int qb = axis;
        int k[2], n = 0;
        float v[2], nacc[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const bool other = ((q & qb) != 0) == (dir < 0);
          if (other) {
            k[n & 1] = half | (q << 1);
            v[n & 1] = acc[q];
            ++n;
          }
          nacc[q] = other ? acc[q ^ qb] : 0.f;
        }
        flush_n(run, 2, k, v);
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[q] = nacc[q];
      }
      cur = kk;
    }
    acc[0] = acc[0] + w.x * dv;
    acc[1] = acc[1] + w.y * dv;
    acc[2] = acc[2] + w.z * dv;
    acc[3] = acc[3] + w.w * dv;
    run = pt;
  }
  {
    const int k[4] = {half, half | 2, half | 4, half | 6};
    flush_n(run, 4, k, acc);
  }
}

// the lane id computed where it is used (volatile: not hoisted out of the tile loop).
// k_mlp_dx runs at its register cap: the staging's per-lane LDS addresses, kept live
// across the tile loop, were spilled and each reload waited vmcnt(0) -- behind the
// tile's record / point-gradient stores and corner loads
__device__ __forceinline__ int lane_here() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}

__device__ __forceinline__ void grid_scatter(const nc_grid& G, const Corners& c, const float dc[8], bool valid,
                                             float* reg, int, int, int) {
  const int lane = lane_here(), i = lane & 15, g = lane >> 4;
  grid_scatter_stage(G, c, dc, valid, reg, i, g);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  grid_scatter_flush(G, reg, lane);
}


}  // namespace nc
