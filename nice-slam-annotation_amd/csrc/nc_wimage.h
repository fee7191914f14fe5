// Split-f16 forward weight images, built once per forward in global memory.
//
// k_mlp_fwd's decoders read their weights from LDS as the NetH image (nc_device.h): every
// pts_linears / fc_c matrix as three round-to-nearest f16 planes in swizzled 128-B / 64-B
// rows, the biases, output layer and Fourier B as floats.  Round 5 built that image in the
// prologue of every forward workgroup (global loads, zero fill, 2-byte LDS stores of three
// planes per weight): 5-6 us of the forward's 78 at C2 (round 6 `fwd_copy_prologue` /
// `fwd_no_wimage` ablations: 72-73 us).  Here a few extra workgroups of the kernel that
// precedes k_mlp_fwd on the stream (k_ray_setup, k_points_prep) write the finished image
// for each job to the workspace, whole 16-B chunks at a time (no zero fill: every chunk of
// the image, padding included, is written), and k_mlp_fwd copies it flat into LDS.
//
// Range guard: the image's split is exact only for |w| < RANGE_LIMIT.  Each builder
// workgroup writes one flag word after the image (1 = a weight it split reached the limit
// or is not finite); k_mlp_fwd ORs the WIMG_WGS words into its amax, exactly as the
// in-workgroup build folded max |w| (so the job is then recomputed by k_mlp_fwd_exact).
// Every word is written by one workgroup on every build: no zeroing, no ordering.
#pragma once
#include "nc_device.h"
#include "nc_internal.h"

namespace nc {

#ifndef NC_WIMG_WGS
#define NC_WIMG_WGS 8
#endif
constexpr int WIMG_WGS = NC_WIMG_WGS;  // builder workgroups per job and image (256 threads each)
constexpr int WIMG_THREADS = 256;

template <int KIND>
__host__ __device__ constexpr int wimg_bytes() { return NetH<KIND>::BYTES; }
constexpr int wimg_max(int a, int b) { return a > b ? a : b; }
// bytes per job in the workspace: the largest image + the flag words, 256-B aligned
constexpr int64_t WIMG_STRIDE =
    ((int64_t)wimg_max(wimg_max(wimg_bytes<K_COARSE>(), wimg_bytes<K_MID>()), wimg_max(wimg_bytes<K_FINE>(), wimg_bytes<K_COLOR>())) +
     4 * WIMG_WGS + 255) & ~int64_t(255);

// one job's weight pointers, selected out of the by-value WImgCtx by constant indices only
// (a reference to wi.dec[j] with a dynamic j makes the compiler copy the kernel argument
// block to scratch: 752 B per lane in k_ray_setup)
struct WSrc {
  const float* lin_w[5];
  const float* lin_b[5];
  const float* fc_w[5];
  const float* fc_b[5];
  const float* fourier_B;
  const float* out_w;
  const float* out_b;
};

// float e (< F32_FLOATS) of the image's f32 part
template <int KIND>
__device__ __forceinline__ float wimg_f32(const WSrc& P, int e) {
  using N = Net<KIND>;
  using H = NetH<KIND>;
  if (e < H::BC) {
    const int L = e >> 5;
    const float* b = L == 0 ? P.lin_b[0] : L == 1 ? P.lin_b[1] : L == 2 ? P.lin_b[2] : L == 3 ? P.lin_b[3] : P.lin_b[4];
    return b[e & 31];
  }
  if (e < H::WO) {  // XYZ only (BC == WO otherwise)
    const int r = e - H::BC, L = r >> 5;
    const float* b = L == 0 ? P.fc_b[0] : L == 1 ? P.fc_b[1] : L == 2 ? P.fc_b[2] : L == 3 ? P.fc_b[3] : P.fc_b[4];
    return b[r & 31];
  }
  if (e < H::BO) return (e - H::WO) < N::NOUT * HID ? P.out_w[e - H::WO] : 0.f;
  if (e < H::FB) return (e - H::BO) < N::NOUT ? P.out_b[e - H::BO] : 0.f;
  if constexpr (N::XYZ) {
    const int r = e - H::FB;
    if (r < 3 * EMBP) {
      const int k = r / EMBP, m = r - k * EMBP;
      return m < EMB ? P.fourier_B[k * EMB + m] : 0.f;
    }
  }
  return 0.f;
}

// Workgroup `slice` of WIMG_WGS writes its share of job's image `img` (16-B chunks, grid-
// strided over the WIMG_WGS workgroups) and its flag word.  Items: the f32 part by 4
// floats, then one item per
// (matrix, row, chunk g): the 8 weights W[o][32 kb + feat_of(j, g)] (row = 32 kb + o)
// split into h, md, l3 (load_weights_h's arithmetic) and stored as the hi chunk, the lo
// chunk and the third-plane chunk of that row.
template <int KIND>
__device__ __forceinline__ void wimg_build(const WSrc& P, char* img, int slice) {
  using N = Net<KIND>;
  using H = NetH<KIND>;
  constexpr int NF4 = H::F32_FLOATS / 4;
  constexpr int NMAT = N::XYZ ? 10 : 5;
  float amax = 0.f;
  const int gt = slice * WIMG_THREADS + (int)threadIdx.x;  // this thread's items: it = gt (mod STRIDE)
  constexpr int STRIDE = WIMG_WGS * WIMG_THREADS;
  for (int it = gt; it < NF4; it += STRIDE) {
    float4 v;
    v.x = wimg_f32<KIND>(P, 4 * it + 0);
    v.y = wimg_f32<KIND>(P, 4 * it + 1);
    v.z = wimg_f32<KIND>(P, 4 * it + 2);
    v.w = wimg_f32<KIND>(P, 4 * it + 3);
    reinterpret_cast<float4*>(img)[it] = v;
  }
  // matrix by matrix (m a constant after unrolling: its pointer and shape are scalars; a
  // per-lane m made the compiler index the pointers through a scratch array)
  int base = NF4;  // global item number of the matrix's first item
#pragma unroll
  for (int m = 0; m < NMAT; ++m) {
    const int rows = m < 5 ? H::kin(m) : N::CD;
    const float* W = m == 0 ? P.lin_w[0] : m == 1 ? P.lin_w[1] : m == 2 ? P.lin_w[2] : m == 3 ? P.lin_w[3]
                   : m == 4 ? P.lin_w[4] : m == 5 ? P.fc_w[0] : m == 6 ? P.fc_w[1] : m == 7 ? P.fc_w[2]
                   : m == 8 ? P.fc_w[3] : P.fc_w[4];
    const int off = m < 5 ? H::lin_off(m) : H::fc_off(m - 5);
    const int off3 = m < 5 ? H::lin3_off(m) : H::fc3_off(m - 5);
    for (int it = base + (((gt - base) % STRIDE) + STRIDE) % STRIDE; it < base + 4 * rows; it += STRIDE) {
      const int q = it - base, g = q & 3, r = q >> 2;
      const int o = r & 31, kb = r >> 5;
      half8 h8, m8, l8;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int cp = 32 * kb + feat_of(j, g);
        float v;
        if (m < 5) {
          const int c = N::real_col(m, cp);
          v = c >= 0 ? W[o * N::in_real(m) + c] : 0.f;
        } else {
          v = W[o * N::CD + cp];
        }
        amax = fmaxf(amax, fabsf(v));  // split-f16 range guard (RANGE_LIMIT)
        // three round-to-nearest planes: v = h + 2^-11 (md + l3), the residuals exact in f32
        const _Float16 h = (_Float16)v;
        const float r1 = (v - (float)h) * SPLIT_SCALE;
        const _Float16 md = (_Float16)r1;
        h8[j] = h;
        m8[j] = md;
        l8[j] = (_Float16)(r1 - (float)md);
      }
      *reinterpret_cast<half8*>(img + off + r * HROW + hchunk(r, g, 0)) = h8;
      *reinterpret_cast<half8*>(img + off + r * HROW + hchunk(r, g, 1)) = m8;
      *reinterpret_cast<half8*>(img + off3 + r * HROW3 + hchunk3(r, g)) = l8;
    }
    base += 4 * rows;
  }
  const bool flag = __syncthreads_or(!(amax < RANGE_LIMIT));
  if (threadIdx.x == 0) reinterpret_cast<uint32_t*>(img + H::BYTES)[slice] = flag ? 1u : 0u;
}

// k_mlp_dx's f32 image (Net<KIND, PADW_BWD>: what load_weights<KIND, PADW_BWD> writes
// into LDS), built by the same forward (the backward reads the weights the forward used,
// as the reference's saved tensors): float4 items, region by region (each region's
// pointer a constant), padding columns written as zeros.  The tail (biases, output
// layer, Fourier B) has the f32-part layout of the split image, at N::BL.
constexpr int DXIMG_FLOATS = wimg_max(wimg_max(Net<K_COARSE, PADW_BWD>::WEIGHTS, Net<K_MID, PADW_BWD>::WEIGHTS),
                                      wimg_max(Net<K_FINE, PADW_BWD>::WEIGHTS, Net<K_COLOR, PADW_BWD>::WEIGHTS));
constexpr int64_t DXIMG_STRIDE = ((int64_t)DXIMG_FLOATS * 4 + 255) & ~int64_t(255);

template <int KIND>
__device__ __forceinline__ void dximg_build(const WSrc& P, float* img, int slice) {
  using N = Net<KIND, PADW_BWD>;
  constexpr int STRIDE = WIMG_WGS * WIMG_THREADS;
  constexpr int NMAT = N::XYZ ? 10 : 5;
  const int gt = slice * WIMG_THREADS + (int)threadIdx.x;
  int base = 0;  // item (float4) number of the region's first item
#pragma unroll
  for (int m = 0; m < NMAT; ++m) {
    const int ld = m < 5 ? N::lin_ld(m) : N::LDC;
    const int off = m < 5 ? N::lin_off(m) : N::WC + (m - 5) * HID * N::LDC;
    const int n4 = HID * ld / 4;
    const float* W = m == 0 ? P.lin_w[0] : m == 1 ? P.lin_w[1] : m == 2 ? P.lin_w[2] : m == 3 ? P.lin_w[3]
                   : m == 4 ? P.lin_w[4] : m == 5 ? P.fc_w[0] : m == 6 ? P.fc_w[1] : m == 7 ? P.fc_w[2]
                   : m == 8 ? P.fc_w[3] : P.fc_w[4];
    for (int it = base + (((gt - base) % STRIDE) + STRIDE) % STRIDE; it < base + n4; it += STRIDE) {
      const int e = 4 * (it - base), o = e / ld, c0 = e - o * ld;
      float v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int c = c0 + k;
        if (m < 5) {
          const int rc = c < (m == 0 ? N::IN0 : m == 3 ? N::IN3 : HID) ? N::real_col(m, c) : -1;
          v[k] = rc >= 0 ? W[o * N::in_real(m) + rc] : 0.f;
        } else {
          v[k] = c < N::CD ? W[o * N::CD + c] : 0.f;
        }
      }
      reinterpret_cast<float4*>(img + off)[it - base] = float4{v[0], v[1], v[2], v[3]};
    }
    base += n4;
  }
  // the tail [BL, WEIGHTS): N::BL is a multiple of 4 floats
  constexpr int T4 = (N::WEIGHTS - N::BL) / 4;
  for (int it = base + (((gt - base) % STRIDE) + STRIDE) % STRIDE; it < base + T4; it += STRIDE) {
    const int e = 4 * (it - base);
    float4 v;
    v.x = wimg_f32<KIND>(P, e + 0);
    v.y = wimg_f32<KIND>(P, e + 1);
    v.z = wimg_f32<KIND>(P, e + 2);
    v.w = wimg_f32<KIND>(P, e + 3);
    reinterpret_cast<float4*>(img + N::BL)[e / 4] = v;
  }
}

// builder workgroup b (0 .. n_jobs * wgs_per_job) of a kernel's extra workgroups
__device__ __forceinline__ void wimg_block(const WImgCtx& w, int b) {
  const int j = b / w.wgs_per_job, slice = b - j * w.wgs_per_job;
  if (j >= w.n_jobs) return;
  const int kind = j == 0 ? w.kind[0] : (j == 1 ? w.kind[1] : w.kind[2]);
  auto sel = [j](const float* a, const float* b, const float* c) { return j == 0 ? a : (j == 1 ? b : c); };
  WSrc P;
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    P.lin_w[k] = sel(w.dec[0].lin_w[k], w.dec[1].lin_w[k], w.dec[2].lin_w[k]);
    P.lin_b[k] = sel(w.dec[0].lin_b[k], w.dec[1].lin_b[k], w.dec[2].lin_b[k]);
    P.fc_w[k] = sel(w.dec[0].fc_w[k], w.dec[1].fc_w[k], w.dec[2].fc_w[k]);
    P.fc_b[k] = sel(w.dec[0].fc_b[k], w.dec[1].fc_b[k], w.dec[2].fc_b[k]);
  }
  P.fourier_B = sel(w.dec[0].fourier_B, w.dec[1].fourier_B, w.dec[2].fourier_B);
  P.out_w = sel(w.dec[0].out_w, w.dec[1].out_w, w.dec[2].out_w);
  P.out_b = sel(w.dec[0].out_b, w.dec[1].out_b, w.dec[2].out_b);
  if (slice >= WIMG_WGS) {  // k_mlp_dx's f32 image
    float* dimg = w.dximg + (int64_t)j * (DXIMG_STRIDE / 4);
    switch (kind) {
      case K_COARSE: dximg_build<K_COARSE>(P, dimg, slice - WIMG_WGS); break;
      case K_MID: dximg_build<K_MID>(P, dimg, slice - WIMG_WGS); break;
      case K_FINE: dximg_build<K_FINE>(P, dimg, slice - WIMG_WGS); break;
      default: dximg_build<K_COLOR>(P, dimg, slice - WIMG_WGS); break;
    }
    return;
  }
  char* img = w.img + (int64_t)j * WIMG_STRIDE;
  switch (kind) {
    case K_COARSE: wimg_build<K_COARSE>(P, img, slice); break;
    case K_MID: wimg_build<K_MID>(P, img, slice); break;
    case K_FINE: wimg_build<K_FINE>(P, img, slice); break;
    default: wimg_build<K_COLOR>(P, img, slice); break;
  }
}

}  // namespace nc
