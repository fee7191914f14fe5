// nc_grid.hip -- the forward trilinear feature lookups (k_grid_gather).  Their
// backward (coordinate gradient + grid scatter, nc_grid.h) runs inside k_mlp_dx.
#include "nc_device.h"
#include "nc_internal.h"

namespace nc {

__device__ __forceinline__ Job pick_job3(const Job (&jobs)[MAX_JOBS], unsigned y) {
  return y == 0 ? jobs[0] : (y == 1 ? jobs[1] : jobs[2]);
}

// Sparse gradient rows (nc_grid.grad_rows, ABI v5): the first lookup that touches an
// in-bounds voxel claims it -- compare-and-swap -1 -> -2 on the map entry -- and
// appends the voxel to its wavefront's shard list (one counter atomic per wavefront,
// spread over CLAIM_SHARDS counters).  k_rows_compact (nc_sparse.hip) then gives the
// claims contiguous rows after the existing ones, points the map at them and zeroes
// them.  The backward (nc_grid.h grid_scatter) accumulates into rows[voxel].
__device__ __forceinline__ void claim_row(const MlpCtx& ctx, const nc_grid& G, const Corners& co, int k) {
  const bool in = (co.inb >> k) & 1u;
  const int64_t x = co.x0 + (k & 1), y = co.y0 + ((k >> 1) & 1), z = co.z0 + (k >> 2);
  const int64_t v = in ? (z * G.dims[1] + y) * G.dims[2] + x : 0;
  bool won = false;
  if (in && __hip_atomic_load(G.grad_rows + v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == -1)
    won = atomicCAS(G.grad_rows + v, -1, -2) == -1;
  const uint64_t m = __ballot(won);
  if (m == 0) return;
  const int leader = __builtin_ctzll(m);
  const int lane = __lane_id();
  const int shard = (int)(((int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) % CLAIM_SHARDS);
  int32_t* cnt = ctx.claim_cnt + blockIdx.y * CLAIM_SHARDS + shard;
  int base = 0;
  if (lane == leader) base = atomicAdd(cnt, (int)__builtin_popcountll(m));
  base = __shfl(base, leader);
  if (!won) return;
  const int64_t slot = base + (int64_t)__builtin_popcountll(m & ((uint64_t(1) << lane) - 1));
  if (slot < ctx.claim_cap)  // (by construction: claim_cap covers every lane of the shard's waves)
    ctx.claim_tmp[((int64_t)blockIdx.y * CLAIM_SHARDS + shard) * ctx.claim_cap + slot] = v;
}

// ---------------------------------------------------------------------------
// Forward trilinear lookups (MLP.sample_grid_feature, decoder.py:179-188, and the
// fine decoder's no-grad grid_middle lookup, :196-202) for every (point, job), as
// their own high-occupancy kernel so the decoder kernel reads contiguous features.
// Thread = (point, GATHER_CH-channel chunk q): chunks 0 .. 32/GATHER_CH - 1 sample the
// job's own grid, the next ones (fine decoder) grid_middle -- unless the middle
// decoder of the same stage has the same bound, whose lookup is then written to both
// (MlpCtx::share_mid).  Corners and weights are make_corners (bit-identical to ATen's
// grid_sampler_3d); channels accumulate corner by corner without FMA.
// ---------------------------------------------------------------------------
#ifndef NC_GATHER_CH
#define NC_GATHER_CH 4
#endif
constexpr int GATHER_CH = NC_GATHER_CH;          // channels per thread (4 or 8)
constexpr int GATHER_V4 = GATHER_CH / 4;         // float4s per corner and thread
constexpr int GATHER_CHUNKS = 32 / GATHER_CH;    // threads per 32-channel lookup
constexpr int GATHER_LG = GATHER_CH == 4 ? 3 : 2;
static_assert(GATHER_CH == 4 || GATHER_CH == 8, "gather chunk width");

__global__ void __launch_bounds__(256) k_grid_gather(const MlpCtx ctx) {
  const unsigned y = blockIdx.y;
  const Job job = y == 0 ? ctx.jobs[0] : (y == 1 ? ctx.jobs[1] : ctx.jobs[2]);
  const int lg = (job.kind == K_FINE && !ctx.share_mid) ? GATHER_LG + 1 : GATHER_LG;  // log2(chunks per point)
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t p = t >> lg;
  if (ctx.zero_fill) {  // the backward's gradient buffer, zeroed beside the gathers (stores last:
                        // nothing waits on them in this thread)
    const int64_t nthr = (int64_t)gridDim.x * blockDim.x * gridDim.y;
    const int64_t tid = (int64_t)blockIdx.y * gridDim.x * blockDim.x + t;
    if (p >= ctx.P) {
      for (int64_t z = tid; z < ctx.zero_n4; z += nthr) ctx.zero_fill[z] = float4{0.f, 0.f, 0.f, 0.f};
      return;
    }
  }
  if (p >= ctx.P) return;
  const int q = (int)(t & ((1 << lg) - 1));
  const bool own = q < GATHER_CHUNKS;
  const int gk = own ? job.kind : K_MID;
  // field-wise constant-index selects (a dynamic index into the kernel-argument
  // grid table would go through scratch)
  nc_grid G;
  G = gk == 0 ? ctx.grids[0] : gk == 1 ? ctx.grids[1] : gk == 2 ? ctx.grids[2] : ctx.grids[3];
  const float4 n = ctx.xyz[(int64_t)job.slot * ctx.P + p];
  const float xyz[3] = {n.x, n.y, n.z};
  Corners co;
  make_corners(G, xyz, co);
  const int c0 = GATHER_CH * (q & (GATHER_CHUNKS - 1));
  const bool vec = grid_vec_ok(G);
  const int64_t sC = G.stride[0];
  float4 v[8][GATHER_V4];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
#pragma unroll
    for (int h = 0; h < GATHER_V4; ++h) {
      const float* base = G.data + corner_off(G, co, k) + (vec ? c0 + 4 * h : (c0 + 4 * h) * sC);
      if (vec) {
        v[k][h] = *reinterpret_cast<const float4*>(base);
      } else {
        v[k][h] = float4{base[0], base[sC], base[2 * sC], base[3 * sC]};
      }
    }
  }
  float4 o[GATHER_V4];
#pragma unroll
  for (int h = 0; h < GATHER_V4; ++h) {
    o[h] = float4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const bool in = (co.inb >> k) & 1u;
      const float w = co.w[k];
      o[h].x = o[h].x + (in ? v[k][h].x * w : 0.f);
      o[h].y = o[h].y + (in ? v[k][h].y * w : 0.f);
      o[h].z = o[h].z + (in ? v[k][h].z * w : 0.f);
      o[h].w = o[h].w + (in ? v[k][h].w * w : 0.f);
    }
    *reinterpret_cast<float4*>(ctx.cfeat + job.c_off + p * job.c_stride + GATHER_CH * q + 4 * h) = o[h];
  }
  if (ctx.claim_rows && own && G.grad_rows) {  // sparse gradient rows: chunk q claims corners q, q + CHUNKS, ..
#pragma unroll
    for (int k = 0; k < 8 / GATHER_CHUNKS; ++k) claim_row(ctx, G, co, q + k * GATHER_CHUNKS);
  }
  if (ctx.jac && own) {  // NC_SAVE_POINT_JACOBIAN: d features / d (ix, iy, iz) of these channels
#pragma unroll
    for (int h = 0; h < GATHER_V4; ++h) {
      float4 j[3] = {float4{0.f, 0.f, 0.f, 0.f}, float4{0.f, 0.f, 0.f, 0.f}, float4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int xb = k & 1, yb = (k >> 1) & 1, zb = k >> 2;
        const bool in = (co.inb >> k) & 1u;
        const float sx = in ? (xb ? 1.f : -1.f) * co.wy[yb] * co.wz[zb] : 0.f;
        const float sy = in ? (yb ? 1.f : -1.f) * co.wx[xb] * co.wz[zb] : 0.f;
        const float sz = in ? (zb ? 1.f : -1.f) * co.wx[xb] * co.wy[yb] : 0.f;
        const float4 a = v[k][h];
        j[0].x = j[0].x + sx * a.x; j[0].y = j[0].y + sx * a.y; j[0].z = j[0].z + sx * a.z; j[0].w = j[0].w + sx * a.w;
        j[1].x = j[1].x + sy * a.x; j[1].y = j[1].y + sy * a.y; j[1].z = j[1].z + sy * a.z; j[1].w = j[1].w + sy * a.w;
        j[2].x = j[2].x + sz * a.x; j[2].y = j[2].y + sz * a.y; j[2].z = j[2].z + sz * a.z; j[2].w = j[2].w + sz * a.w;
      }
      float* dst = ctx.jac + ((int64_t)job.slot * ctx.P + p) * 96 + GATHER_CH * q + 4 * h;
#pragma unroll
      for (int a = 0; a < 3; ++a) *reinterpret_cast<float4*>(dst + 32 * a) = j[a];
    }
  }
  if (ctx.share_mid && y == 1) {  // the fine decoder's no-grad grid_middle lookup is this one
#pragma unroll
    for (int h = 0; h < GATHER_V4; ++h)
      *reinterpret_cast<float4*>(ctx.cfeat + ctx.jobs[0].c_off + p * ctx.jobs[0].c_stride + 32 + GATHER_CH * q + 4 * h) = o[h];
  }
  if (ctx.zero_fill) {
    const int64_t nthr = (int64_t)gridDim.x * blockDim.x * gridDim.y;
    const int64_t tid = (int64_t)blockIdx.y * gridDim.x * blockDim.x + t;
    for (int64_t z = tid; z < ctx.zero_n4; z += nthr) ctx.zero_fill[z] = float4{0.f, 0.f, 0.f, 0.f};
  }
}

int launch_grid_gather(const MlpCtx& c, hipStream_t s) {
  const int64_t threads = c.P * 2 * GATHER_CHUNKS;  // the widest job (fine: two lookups per point)
  hipLaunchKernelGGL(k_grid_gather, dim3((unsigned)((threads + 255) / 256), c.n_jobs), dim3(256), 0, s, c);
  return (int)hipGetLastError();
}


}  // namespace nc
