// nc_rays.hip — per-ray stages of Renderer.render_batch_ray on gfx950.
//
// One wavefront per ray, lane = sample (S = N_samples + N_surface <= 64):
//   k_ray_setup      Renderer.py:120-231  near/far, bbox slab test, stratified +
//                    surface samples, 64-lane bitonic merge-sort, float64 points
//   k_composite_fwd  common.py:215-256 (occupancy=True) + Renderer.py:87 mask:
//                    alpha, exclusive transmittance product by a wavefront scan,
//                    depth / variance (float64) and colour
//   k_composite_bwd  its autograd backward: d occupancy and d rgb per sample,
//                    the transmittance term by a reverse affine wavefront scan
//   k_loss           the fused Mapper / Tracker rendering loss + per-ray derivatives
//   k_ray_grads      d rays_o / d rays_d from the per-decoder point gradients
//   k_param_reduce   sum of the per-workgroup weight-gradient slabs
// All floating-point expressions keep the reference's association order and the
// file is compiled with -ffp-contract=off, so the sample depths and points are
// bit-identical to the CPU reference.
#include <math.h>

#include "nc_device.h"
#include "nc_internal.h"
#include "nc_wimage.h"

namespace nc {

constexpr int RAY_WAVES = 4;  // rays per 256-thread workgroup

__global__ void __launch_bounds__(1024) k_depth_max(const float* gt, const uint8_t* valid, int64_t n, float* out) {
  __shared__ float red[16];
  float m = -INFINITY;
  for (int64_t k = threadIdx.x; k < n; k += blockDim.x) {
    if (valid && !valid[k]) continue;  // dropped rays (ray_valid) are not in the batch
    const float v = gt[k];
    m = (v > m || isnan(v)) ? v : m;
  }
  for (int o = 32; o > 0; o >>= 1) {
    const float v = __shfl_xor(m, o);
    m = (v > m || isnan(v)) ? v : m;
  }
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    float r = red[0];
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) r = (red[w] > r || isnan(red[w])) ? red[w] : r;
    *out = r;
  }
}

__device__ __forceinline__ bool gt_nan_last(double a, double b) {  // a > b, NaN largest (torch.sort)
  return (isnan(a) && !isnan(b)) || a > b;
}

__device__ __forceinline__ double max_nan(double a, double b) { return (a > b || isnan(a)) ? a : b; }
__device__ __forceinline__ double min_nan(double a, double b) { return (a < b || isnan(a)) ? a : b; }

// grid: wi.n_jobs * wi.wgs_per_job workgroups that build the decoders' weight images
// (nc_wimage.h), the ray workgroups, then ray_fill_wgs(c) fill workgroups
__host__ __device__ inline unsigned ray_fill_wgs(const RayCtx& c) {
  return (c.zero_fill && c.zero_lo4 > 0) ? (unsigned)c.zero_wgs_setup : 0u;
}

__global__ void __launch_bounds__(256) k_ray_setup(const RayCtx c, const WImgCtx wi) {
  // the weight-image builders first (dispatched with the rays, not after the fill)
  const unsigned nbuild = (unsigned)(wi.n_jobs * wi.wgs_per_job);
  if (blockIdx.x < nbuild) {
    wimg_block(wi, (int)blockIdx.x);
    return;
  }
  const unsigned blk = blockIdx.x - nbuild;
  const unsigned nb = (unsigned)((c.N + RAY_WAVES - 1) / RAY_WAVES);  // ray workgroups
  if (blk >= nb) {  // the first part of the gradient buffer's zero fill (RayCtx::zero_lo4)
    const int64_t nthr = (int64_t)c.zero_wgs_setup * blockDim.x;
    for (int64_t z = (int64_t)(blk - nb) * blockDim.x + threadIdx.x; z < c.zero_lo4; z += nthr)
      c.zero_fill[z] = float4{0.f, 0.f, 0.f, 0.f};
    return;
  }
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blk * RAY_WAVES + (threadIdx.x >> 6);
  if (blk == 0 && threadIdx.x < MAX_JOBS && c.range_flag) c.range_flag[threadIdx.x] = 0u;  // for k_mlp_fwd
  if (blk == 0 && threadIdx.x == 0 && c.fuse_bwd) *c.loss_count = 0u;  // k_composite_fwd_loss's done counter
  // this ray's inputs first: their loads overlap the batch-max loop below
  const bool live = r < c.N;
  const int64_t rr = live ? r : 0;
  double o[3], d[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    o[k] = (double)c.rays_o[rr * 3 + k];
    d[k] = (double)c.rays_d[rr * 3 + k];
  }
  const float gd_in = (c.gt_depth && c.N > 0) ? c.gt_depth[rr] : 0.f;
  // the per-lane sample inputs too (clamped indices, used below by lane range): a load
  // under a branch of its only use is issued alone and waited for
  const float t_str = c.t_strat[lane < c.n_strat ? lane : 0];
  const double t_srf = c.n_surf > 0 ? c.t_surf[lane >= c.n_strat && lane < c.n_strat + c.n_surf ? lane - c.n_strat : 0] : 0.0;
  const int xl = lane - c.n_strat - c.n_surf;
  const double z_ex = c.n_extra > 0 ? c.z_extra[rr * c.n_extra + (xl >= 0 && xl < c.n_extra ? xl : 0)] : 0.0;
  const float t_rnd = c.t_rand ? c.t_rand[rr * c.n_strat + (lane < c.n_strat ? lane : 0)] : 0.f;
  const float dmax_arg = *(c.depth_max ? c.depth_max : reinterpret_cast<const float*>(c.z));  // when !dmax_local
  const bool ok = ray_ok(c, rr);  // a dropped ray's samples stay finite: they feed the decoders
  float dmax_blk = 0.f;
  if (c.dmax_local) {  // torch.max(gt_depth) over the whole batch, by every workgroup (N small)
    __shared__ float red[RAY_WAVES];
    float m = -INFINITY;
    // 4 strides at a time, every load unconditional (clamped index; without a mask the
    // flag byte is read from the depths and ignored) so all 8 are in flight together
    constexpr int U = 4;
    for (int64_t k0 = threadIdx.x; k0 < c.N; k0 += U * blockDim.x) {
      float v[U];
      uint8_t f[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t k = k0 + u * blockDim.x < c.N ? k0 + u * blockDim.x : c.N - 1;
        v[u] = c.gt_depth[k];
        f[u] = *(c.valid ? c.valid + k : reinterpret_cast<const uint8_t*>(c.gt_depth));
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {  // in k order; dropped rays (ray_valid) are not in the batch
        const bool keep = k0 + u * blockDim.x < c.N && (!c.valid || f[u]);
        m = keep && (v[u] > m || isnan(v[u])) ? v[u] : m;
      }
    }
    for (int o = 32; o > 0; o >>= 1) {
      const float v = __shfl_xor(m, o);
      m = (v > m || isnan(v)) ? v : m;
    }
    if (lane == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    m = red[0];
    for (int w = 1; w < RAY_WAVES; ++w) m = (red[w] > m || isnan(red[w])) ? red[w] : m;
    dmax_blk = m;
  }
  if (!live) return;
  // Renderer.py:139-152: far_bb = min_axis(max(t0, t1)) + 0.01 (no grad, float64)
  double far_bb = 0.0;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const double t0 = (c.bound[k][0] - o[k]) / d[k];
    const double t1 = (c.bound[k][1] - o[k]) / d[k];
    const double mk = max_nan(t0, t1);
    far_bb = (k == 0) ? mk : min_nan(far_bb, mk);
  }
  far_bb = far_bb + 0.01;
  const bool has_depth = c.n_surf > 0 || c.gt_depth != nullptr;
  double far = far_bb;
  float gd = 0.f, dmax = 0.f;
  if (has_depth) {
    gd = gd_in;
    dmax = c.dmax_local ? dmax_blk : dmax_arg;
    const double hi = (double)(dmax * 1.2f);  // torch.max(gt_depth*1.2) (float32)
    double v = far_bb < 0.0 ? 0.0 : far_bb;   // torch.clamp(far_bb, 0, hi)
    far = v > hi ? hi : v;
  }
  double z;
  if (lane < c.n_strat) {
    const float t = t_str;
    const float om = 1.0f - t;                               // (1.-t_vals)
    if (!c.lindisp) {
      const float nearw = has_depth ? (gd * 0.01f) * om : 0.01f * om;  // near*(1-t), float32
      z = (double)nearw + far * (double)t;                   // + far*t (float64)
    } else {  // Renderer.py:209: 1./(1./near*(1.-t) + 1./far*t); 1./x is reciprocal(x)*1.
      const float inv_near = has_depth ? 1.0f / (gd * 0.01f) : 100.0f;  // float32 (no depth: 1./0.01 = 100.)
      z = 1.0 / ((double)(inv_near * om) + (1.0 / far) * (double)t);
    }
  } else if (lane < c.n_strat + c.n_surf) {
    const double ts = t_srf;
    if (gd > 0.f) {  // Renderer.py:185-187
      z = (double)(0.95f * gd) * (1.0 - ts) + (double)(1.05f * gd) * ts;
    } else {         // Renderer.py:193-196
      z = 0.001 * (1.0 - ts) + (double)dmax * ts;
    }
  } else if (lane < c.S) {  // importance samples (Renderer.py:248: sorted with the rest)
    z = z_ex;
  } else {
    z = INFINITY;
  }
  if (c.t_rand) {  // Renderer.py:211-219: mids of neighbours, z = lower + (upper - lower) * t_rand
    const double zp = __shfl_up(z, 1), zn = __shfl_down(z, 1);
    if (lane < c.n_strat) {
      const double lower = lane > 0 ? .5 * (z + zp) : z;
      const double upper = lane < c.n_strat - 1 ? .5 * (zn + z) : z;
      z = lower + (upper - lower) * (double)t_rnd;
    }
  }
  if (c.n_surf > 0 || c.n_extra > 0) {  // Renderer.py:222-224 / :248 torch.sort (bitonic, 64 lanes)
#pragma unroll
    for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
      for (int j = k >> 1; j > 0; j >>= 1) {
        const double other = xor_lane(z, j);
        const bool up = (lane & k) == 0;
        const bool lower = (lane & j) == 0;
        const bool take_min = (lower == up);
        const bool zg = gt_nan_last(z, other);
        z = take_min ? (zg ? other : z) : (zg ? z : other);
      }
    }
  }
  if (!ok && !isfinite(z)) z = 0.0;
  if (lane < c.S) {
    const int64_t p = r * c.S + lane;
    c.z[p] = z;
    if (c.z_out) c.z_out[p] = z;
    double pt[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      pt[k] = o[k] + d[k] * z;  // Renderer.py:227-228
      if (!ok && !isfinite(pt[k])) pt[k] = 0.0;
      c.pts[p * 3 + k] = pt[k];
    }
    c.pf[p] = float4{(float)pt[0], (float)pt[1], (float)pt[2], 0.f};
    for (int j = 0; j < c.n_jobs; ++j) {
      float n[3];
      normalize_pt(pt, j == 0 ? c.job_bound[0] : (j == 1 ? c.job_bound[1] : c.job_bound[2]), n);
      c.xyz[(int64_t)j * c.P + p] = float4{n[0], n[1], n[2], 0.f};
    }
  }
}

// points mode (NICE.forward on caller points): the same per-point prologue
__global__ void __launch_bounds__(256) k_points_prep(const MlpCtx m, const WImgCtx wi, float4* xyz, float4* pf) {
  const unsigned nbuild = (unsigned)(wi.n_jobs * wi.wgs_per_job);
  if (blockIdx.x < nbuild) {  // the decoders' weight images (nc_wimage.h)
    wimg_block(wi, (int)blockIdx.x);
    return;
  }
  const int64_t p = (int64_t)(blockIdx.x - nbuild) * blockDim.x + threadIdx.x;
  if (p < MAX_JOBS && m.range_flag) m.range_flag[p] = 0u;  // for k_mlp_fwd
  if (p >= m.P) return;
  double pt[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) pt[k] = m.pts[p * 3 + k];
  pf[p] = float4{(float)pt[0], (float)pt[1], (float)pt[2], 0.f};
  for (int j = 0; j < m.n_jobs; ++j) {
    const Job job = j == 0 ? m.jobs[0] : (j == 1 ? m.jobs[1] : m.jobs[2]);
    const nc_decoder_params& D = job.kind == 0 ? m.dec[0] : job.kind == 1 ? m.dec[1] : job.kind == 2 ? m.dec[2] : m.dec[3];
    float n[3];
    normalize_pt(pt, D.bound, n);
    xyz[(int64_t)j * m.P + p] = float4{n[0], n[1], n[2], 0.f};
  }
}

// strict in-bound mask of Renderer.py:63-66 against the renderer bound
// (the three coordinates loaded first and the tests combined without short-circuit: with
// && each later load sits in a branch of its own and is waited for alone)
__device__ __forceinline__ bool in_bound(const double* p, const double (&b)[3][2]) {
  const double x = p[0], y = p[1], z = p[2];
  return (x < b[0][1]) & (x > b[0][0]) & (y < b[1][1]) & (y > b[1][0]) & (z < b[2][1]) & (z > b[2][0]);
}

struct SampleState {
  double z;
  float a, q, T, w;
  float rgb[3];
  bool inb;
  float dist, nrm, sig, e;  // density mode (iMAP*)
};

// shared by forward and backward: alpha, exclusive product T, weights
__device__ __forceinline__ void sample_state(const RayCtx& c, int64_t r, int lane, SampleState& s) {
  const bool act = lane < c.S;
  const int64_t p = r * c.S + (act ? lane : 0);
  const double zl = c.z[p];  // p is clamped: loaded unconditionally, then selected
  s.z = act ? zl : 0.0;
  // every per-sample load of the state unconditional, so they issue together (a load under
  // a branch, even a uniform one, is waited for before the loads after the branch)
  const float* ob = c.occ ? c.occ : reinterpret_cast<const float*>(c.z);
  const float oa = ob[(int64_t)(c.occ_a >= 0 ? c.occ_a : 0) * c.P + p];
  const float obv = ob[(int64_t)(c.occ_b >= 0 ? c.occ_b : 0) * c.P + p];
  const float occ_a = c.occ_a >= 0 ? oa : 0.f;
  const float occ_ab = occ_a + obv;  // fine_occ + middle_occ (formed always: a select, not a branch)
  float occ = c.occ_b >= 0 ? occ_ab : occ_a;
  s.inb = in_bound(c.pts + p * 3, c.bound);
  if (!s.inb) occ = 100.f;  // Renderer.py:87
  // colour loaded unconditionally too (from the sample depths when there is none)
  const float* rp = c.has_rgb ? c.rgb + p * 3 : reinterpret_cast<const float*>(c.z + p);
  float rv[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) rv[k] = rp[k];
#pragma unroll
  for (int k = 0; k < 3; ++k) s.rgb[k] = c.has_rgb ? rv[k] : 0.f;
  if (c.density) {  // iMAP*: raw2alpha(raw, dists) = 1 - exp(-relu(raw) * dists) (common.py:232-247)
    const double zn = __shfl_down(s.z, 1);
    s.dist = (lane + 1 < c.S) ? (float)(zn - s.z) : 1e10f;  // dists.float(), 1e10 after the last sample
    const float* d = c.rays_d + r * 3;
    s.nrm = sqrtf(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);  // torch.norm(rays_d)
    s.sig = occ;
    s.e = expf(-(occ > 0.f ? occ : 0.f) * (s.dist * s.nrm));
    s.a = 1.f - s.e;
  } else {
    const float x = 10.f * occ;
    s.a = 1.f / (1.f + expf(-x));          // torch.sigmoid
  }
  s.q = act ? (1.f - s.a) + 1e-10f : 1.f; // (1.-alpha + 1e-10)
  // exclusive prefix product over the wavefront (Hillis-Steele on 64 lanes)
  float incl = s.q;
#pragma unroll
  for (int dlt = 1; dlt < 64; dlt <<= 1) {
    const float v = __shfl_up(incl, dlt);
    if (lane >= dlt) incl = incl * v;
  }
  const float ex = __shfl_up(incl, 1);
  s.T = lane == 0 ? 1.f : ex;
  s.w = act ? s.a * s.T : 0.f;
  if (!act) {
    s.a = 0.f;
    s.rgb[0] = s.rgb[1] = s.rgb[2] = 0.f;
  }
}

__device__ __forceinline__ double wsum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += xor_lane(v, o);
  return v;
}
__device__ __forceinline__ float wsum_f(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += xor_lane(v, o);
  return v;
}

// raw2outputs_nerf_color's outputs of ray r (common.py:248-256): depth, var, colour
__device__ __forceinline__ void composite_fwd_ray(const RayCtx& c, int64_t r, int lane, const SampleState& s,
                                                  double& depth, float (&col)[3]) {
  col[0] = wsum_f(s.w * s.rgb[0]);
  col[1] = wsum_f(s.w * s.rgb[1]);
  col[2] = wsum_f(s.w * s.rgb[2]);
  depth = wsum_d((double)s.w * s.z);
  const double tmp = s.z - depth;
  const double var = wsum_d(lane < c.S ? ((double)s.w * tmp) * tmp : 0.0);
  const bool ok = ray_ok(c, r);  // a dropped ray (ray_valid) reports zeros
  if (c.weights_out && lane < c.S) c.weights_out[r * c.S + lane] = ok ? s.w : 0.f;
  if (lane == 0) {
    c.depth[r] = ok ? depth : 0.0;
    c.var[r] = ok ? var : 0.0;
    c.color[r * 3 + 0] = ok ? col[0] : 0.f;
    c.color[r * 3 + 1] = ok ? col[1] : 0.f;
    c.color[r * 3 + 2] = ok ? col[2] : 0.f;
  }
}

__global__ void __launch_bounds__(256) k_composite_fwd(const RayCtx c) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * RAY_WAVES + (threadIdx.x >> 6);
  if (r >= c.N) return;
  SampleState s;
  sample_state(c, r, lane, s);
  double depth;
  float col[3];
  composite_fwd_ray(c, r, lane, s, depth, col);
}

// composite backward of ray r from the upstream (gD, gV, gC) of its depth / var / colour
// (common.py:215-256 in reverse): writes d loss / d raw of its samples (gocc, grgb)
__device__ __forceinline__ void composite_bwd_core(const RayCtx& c, int64_t r, int lane, const SampleState& s,
                                                   double depth, double gD, double gV, const float (&gC)[3]) {
  const bool act = lane < c.S;
  // var = sum w (z-D)^2, D = sum w z  (common.py:253-255)
  const double tmp = s.z - depth;
  const double gtmp = act ? 2.0 * gV * (double)s.w * tmp : 0.0;
  const double gDt = gD - wsum_d(gtmp);
  float gw = (float)(gDt * s.z) + (float)(gV * tmp * tmp);
  gw = gw + (gC[0] * s.rgb[0] + gC[1] * s.rgb[1] + gC[2] * s.rgb[2]);
  if (!act) gw = 0.f;
  // w = a * T, T_i = prod_{j<i} q_j, q = 1 - a + 1e-10
  const float gT = gw * s.a;
  // S_l = sum_{i>l} gT_i prod_{l<k<i} q_k  -> reverse scan of x -> b_l + c_l x
  float cB = __shfl_down(gT, 1);
  float cC = __shfl_down(s.q, 1);
  if (lane + 1 >= c.S) { cB = 0.f; cC = 0.f; }
#pragma unroll
  for (int dlt = 1; dlt < 64; dlt <<= 1) {
    const float nb = __shfl_down(cB, dlt);
    const float ncc = __shfl_down(cC, dlt);
    if (lane + dlt < 64) {
      cB = cB + cC * nb;
      cC = cC * ncc;
    }
  }
  const float gq = s.T * cB;
  const float ga = gw * s.T - gq;
  float g_occ;
  if (c.density) {
    // alpha = 1 - exp(-relu(sig) * dist * nrm): d alpha = e * (relu'(sig) dsig * dist * nrm + relu(sig) * dist * dnrm)
    const float ge = act ? ga * s.e : 0.f;
    g_occ = s.sig > 0.f ? ge * (s.dist * s.nrm) : 0.f;
    const float gn = wsum_f(act ? (ge * (s.sig > 0.f ? s.sig : 0.f)) * s.dist : 0.f);
    if (lane == 0 && c.gnorm) c.gnorm[r] = gn;
  } else {
    const float gy = (ga * (1.f - s.a)) * s.a;  // sigmoid backward
    g_occ = gy * 10.f;
  }
  if (!s.inb) g_occ = 0.f;
  if (act) {
    const int64_t p = r * c.S + lane;
    c.gocc[p] = g_occ;
    if (c.has_rgb) {
#pragma unroll
      for (int k = 0; k < 3; ++k) c.grgb[p * 3 + k] = gC[k] * s.w;
    }
  }
}

__global__ void __launch_bounds__(256) k_composite_bwd(const RayCtx c) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * RAY_WAVES + (threadIdx.x >> 6);
  if (r >= c.N) return;
  SampleState s;
  sample_state(c, r, lane, s);
  const double depth = wsum_d((double)s.w * s.z);
  double gD = c.g_depth ? c.g_depth[r] : 0.0;
  const double gV = c.g_var ? c.g_var[r] : 0.0;
  float gC[3] = {0.f, 0.f, 0.f};
  if (c.g_color) {
#pragma unroll
    for (int k = 0; k < 3; ++k) gC[k] = c.g_color[r * 3 + k];
  }
  if (c.loss && c.g_loss) {  // the fused loss's contribution (k_loss)
    const double gl = *c.g_loss;
    gD = gD + gl * c.coef_d[r];
    if (c.loss_flags & NC_LOSS_COLOR) {
#pragma unroll
      for (int k = 0; k < 3; ++k) gC[k] = gC[k] + (float)gl * c.coef_c[r * 3 + k];
    }
  }
  if (!ray_ok(c, r)) {  // a dropped ray passes no gradient on (its d raw is exactly 0)
    gD = 0.0;
    gC[0] = gC[1] = gC[2] = 0.f;
  }
  composite_bwd_core(c, r, lane, s, depth, gD, ray_ok(c, r) ? gV : 0.0, gC);
}

// ---------------------------------------------------------------------------
// k_loss -- the rendering loss of the batch and its per-ray derivatives:
//   NC_LOSS_MAPPER  (Mapper.py:603-612)
//     loss = sum_{gt>0} |gt - depth|              (float64)
//            [+ w * sum |gt_c - color|]           (float32 term, NC_LOSS_COLOR)
//   NC_LOSS_TRACKER (Tracker.py:117-131)
//     tmp  = |gt - depth| / sqrt(var + 1e-10)     (var detached)
//     mask = gt > 0 [& tmp < 10 * median(tmp)]    (NC_LOSS_DYNAMIC: handle_dynamic)
//     loss = sum_mask tmp [+ w * sum_mask |gt_c - color|]
// One 1024-thread workgroup.  torch.median's lower median (NaN if any tmp is NaN)
// is a radix select over the float64 bit patterns (tmp >= 0 orders like its bits as
// unsigned integers): 8 passes of an 8-bit LDS histogram over keys formed once into
// LDS (up to 4,096 rays; beyond, tmp is recomputed from depth/var each pass).  Sums
// are per-thread strided partials + a fixed-order tree (deterministic).  The colour sum accumulates in float64 and is rounded once to
// float32 (the reference's float32 sum is pairwise; both are within ~1 ulp of exact).
// The derivatives are autograd's expressions -- AbsBackward's sgn (sgn(0) = sgn(NaN)
// = 0), DivBackward's 1/s, SubBackward's negation, masked rows 0 -- and go to
// coef_d / coef_c, which k_composite_bwd scales by the upstream g_loss.
// ---------------------------------------------------------------------------
constexpr int LOSS_THREADS = 1024;
constexpr int LOSS_KEYS = 4096;  // rays whose median keys are held in LDS (32 KB)
// key of a dropped ray in the cached median keys: a NaN bit pattern, never a real tmp's
constexpr unsigned long long KEY_DROPPED = ~0ull - 1ull;

__device__ __forceinline__ double sgn_d(double x) { return x > 0.0 ? 1.0 : (x < 0.0 ? -1.0 : 0.0); }
__device__ __forceinline__ float sgn_f(float x) { return x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f); }

__device__ __forceinline__ double tracker_tmp(const RayCtx& c, int64_t r, double& diff, double& s) {
  diff = (double)c.loss_depth[r] - c.depth[r];
  s = sqrt(c.var[r] + 1e-10);
  return fabs(diff) / s;
}

__global__ void __launch_bounds__(LOSS_THREADS) k_loss(const RayCtx c) {
  __shared__ unsigned hist[256];
  __shared__ unsigned long long sel_prefix;
  __shared__ long long sel_k;
  __shared__ int any_nan;
  __shared__ double part_d[LOSS_THREADS / 64], part_c[LOSS_THREADS / 64];
  const int tid = threadIdx.x;
  const bool tracker = c.loss == NC_LOSS_TRACKER;
  const bool dyn = tracker && (c.loss_flags & NC_LOSS_DYNAMIC);
  const bool col = (c.loss_flags & NC_LOSS_COLOR) != 0;
  double thr = 0.0;
  if (dyn) {
    // up to LOSS_KEYS rays (the Tracker's batches) the keys are formed once into LDS
    // (~0 marks NaN); beyond, every pass recomputes tmp from depth / var
    __shared__ unsigned long long skey[LOSS_KEYS];
    __shared__ unsigned vpart[LOSS_THREADS / 64];
    const bool cached = c.N <= LOSS_KEYS;
    if (c.valid) {  // the median is over the kept rays only (ray_valid: the compacted batch)
      unsigned cnt = 0;
      for (int64_t r = tid; r < c.N; r += LOSS_THREADS) cnt += c.valid[r] != 0 ? 1u : 0u;
      for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
      if ((tid & 63) == 0) vpart[tid >> 6] = cnt;
      __syncthreads();
    }
    if (tid == 0) {
      long long nv = (long long)c.N;
      if (c.valid) {
        nv = 0;
        for (int w = 0; w < LOSS_THREADS / 64; ++w) nv += vpart[w];
      }
      sel_prefix = 0ull;
      sel_k = (nv - 1) / 2;
      any_nan = 0;
    }
    if (cached) {
      for (int64_t r = tid; r < c.N; r += LOSS_THREADS) {
        const bool okr = ray_ok(c, r);
        double diff, s;
        const double t = tracker_tmp(c, r, diff, s);
        const unsigned long long kt = isnan(t) ? ~0ull : (unsigned long long)__double_as_longlong(t);
        skey[r] = okr ? kt : KEY_DROPPED;  // a select: the flag and the inputs load together
      }
    }
    unsigned long long pmask = 0ull;
    for (int shift = 56; shift >= 0; shift -= 8) {
      if (tid < 256) hist[tid] = 0u;
      __syncthreads();
      const unsigned long long prefix = sel_prefix;
      for (int64_t r = tid; r < c.N; r += LOSS_THREADS) {
        unsigned long long key;
        if (cached) {
          key = skey[r];
          if (key == ~0ull) {
            any_nan = 1;
            continue;
          }
          if (key == KEY_DROPPED) continue;
        } else {
          if (!ray_ok(c, r)) continue;
          double diff, s;
          const double t = tracker_tmp(c, r, diff, s);
          if (isnan(t)) {
            any_nan = 1;
            continue;
          }
          key = (unsigned long long)__double_as_longlong(t);
        }
        if ((key & pmask) == prefix) atomicAdd(&hist[(key >> shift) & 255u], 1u);
      }
      __syncthreads();
      if (tid < 64) {  // wave 0: lane l owns bins 4l..4l+3; find the bin holding rank k
        unsigned h[4];
#pragma unroll
        for (int b = 0; b < 4; ++b) h[b] = hist[4 * tid + b];
        const unsigned tot = h[0] + h[1] + h[2] + h[3];
        unsigned inc = tot;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const unsigned v = __shfl_up(inc, o);
          if (tid >= o) inc += v;
        }
        const long long k = sel_k;
        const long long exc = (long long)(inc - tot);
        if (exc <= k && k < (long long)inc) {
          long long kk = k - exc;
          int b = 0;
          while (b < 3 && kk >= (long long)h[b]) kk -= h[b++];
          sel_k = kk;
          sel_prefix = prefix | ((unsigned long long)(4 * tid + b) << shift);
        }
      }
      __syncthreads();
      pmask |= 255ull << shift;
    }
    const double med = any_nan ? __longlong_as_double(0x7ff8000000000000ll) : __longlong_as_double((long long)sel_prefix);
    thr = 10.0 * med;
  }
  double sd = 0.0, sc = 0.0;
  for (int64_t r = tid; r < c.N; r += LOSS_THREADS) {
    // the ray's inputs loaded first, unconditionally (a load under a branch waits alone);
    // a dropped ray (ray_valid) is masked out of both terms and gets zero coefficients
    const bool ok = ray_ok(c, r);
    const float gt = c.loss_depth[r];
    const double dep = c.depth[r];
    const double vr = c.var[r];
    const float* lcp = col ? c.loss_color + r * 3 : c.loss_depth + r;
    float lc[3], cc[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      lc[k] = lcp[col ? k : 0];
      cc[k] = c.color[r * 3 + k];
    }
    bool m = ok && gt > 0.f;
    double val, coef;
    const double diff = (double)gt - dep;
    if (tracker) {  // tracker_tmp
      const double sdev = sqrt(vr + 1e-10);
      val = fabs(diff) / sdev;
      if (dyn) m = m && (val < thr);
      coef = -(sgn_d(diff) * (1.0 / sdev));
    } else {
      val = fabs(diff);
      coef = -sgn_d(diff);
    }
    sd = m ? sd + val : sd;
    c.coef_d[r] = m ? coef : 0.0;
    if (col) {
      const bool mc = ok && (tracker ? m : true);  // the mapper's colour term is unmasked
      float cf[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const float dc = lc[k] - cc[k];
        sc = mc ? sc + (double)fabsf(dc) : sc;
        cf[k] = mc ? -(c.w_color * sgn_f(dc)) : 0.f;
      }
#pragma unroll
      for (int k = 0; k < 3; ++k) c.coef_c[r * 3 + k] = cf[k];
    }
  }
  sd = wsum_d(sd);
  sc = wsum_d(sc);
  if ((tid & 63) == 0) {
    part_d[tid >> 6] = sd;
    part_c[tid >> 6] = sc;
  }
  __syncthreads();
  if (tid == 0) {
    double d = 0.0, cs = 0.0;
    for (int w = 0; w < LOSS_THREADS / 64; ++w) {
      d += part_d[w];
      cs += part_c[w];
    }
    double loss = d;
    if (col) loss = loss + (double)(c.w_color * (float)cs);
    *c.loss_out = loss;
  }
}

// ---------------------------------------------------------------------------
// k_composite_fwd_loss -- NC_LOSS_MAPPER with a backward to come (RayCtx::fuse_bwd):
// the mapper loss needs no batch-wide statistic, so its per-ray derivatives are known
// as soon as the ray is composited.  One pass per ray does k_composite_fwd, k_loss's
// NC_LOSS_MAPPER terms (the same expressions) and k_composite_bwd for d loss = 1;
// k_mlp_dx multiplies by the actual d loss (MlpCtx::dout_scale), so the backward skips
// k_composite_bwd (and the forward k_loss).  coef_d / coef_c are still written for a
// backward that also receives depth / var / colour gradients.  The loss value, in a
// fixed order (run-to-run identical): each workgroup stores its rays' float64 depth and
// colour sums to loss_part, and the last workgroup to finish (loss_count, zeroed by
// k_ray_setup) sums the partials in block order and applies w_color once to the
// float32-rounded colour total, as k_loss does (Mapper.py:609-612).
// ---------------------------------------------------------------------------
#ifndef NC_FUSED_RAYS
#define NC_FUSED_RAYS 16
#endif
constexpr int FUSED_RAYS = NC_FUSED_RAYS;  // rays (waves) per workgroup: 63 atomics at C2

__global__ void __launch_bounds__(64 * FUSED_RAYS) k_composite_fwd_loss(const RayCtx c) {
  __shared__ double part[FUSED_RAYS][2];
  const unsigned nb = (unsigned)((c.N + FUSED_RAYS - 1) / FUSED_RAYS);  // ray workgroups
  if (blockIdx.x >= nb) {  // the gradient buffer's zero fill on the CUs the rays leave idle
    const int64_t nthr = (int64_t)c.zero_wgs * blockDim.x;
    for (int64_t z = c.zero_lo4 + (int64_t)(blockIdx.x - nb) * blockDim.x + threadIdx.x; z < c.zero_n4; z += nthr)
      c.zero_fill[z] = float4{0.f, 0.f, 0.f, 0.f};
    return;
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t r = (int64_t)blockIdx.x * FUSED_RAYS + wv;
  const bool col_term = (c.loss_flags & NC_LOSS_COLOR) != 0;
  double ld = 0.0, lc = 0.0;
  if (r < c.N) {
    // the loss targets and the ray flag first, with unconditional uses (a load used only
    // in a branch is sunk into it and waited for there, after the compositing)
    const bool ok = ray_ok(c, r);  // a dropped ray (ray_valid) is not in the loss
    const float gt = c.loss_depth[r];
    const float* tcp = col_term ? c.loss_color + r * 3 : c.loss_depth + r;
    float tc[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) tc[k] = tcp[col_term ? k : 0];
    SampleState s;
    sample_state(c, r, lane, s);
    double depth;
    float col[3];
    composite_fwd_ray(c, r, lane, s, depth, col);
    const bool m = ok && gt > 0.f;
    const double diff = (double)gt - depth;
    const double coef = m ? -sgn_d(diff) : 0.0;
    ld = m ? fabs(diff) : 0.0;
    float gC[3];
    const bool use_c = col_term && ok;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const float dc = tc[k] - col[k];
      lc += use_c ? (double)fabsf(dc) : 0.0;  // the mapper's colour term is unmasked
      gC[k] = use_c ? -(c.w_color * sgn_f(dc)) : 0.f;
    }
    if (lane == 0) {
      c.coef_d[r] = coef;
      if (col_term) {
#pragma unroll
        for (int k = 0; k < 3; ++k) c.coef_c[r * 3 + k] = gC[k];
      }
    }
    composite_bwd_core(c, r, lane, s, depth, coef, 0.0, gC);
  }
  if (lane == 0) {
    part[wv][0] = ld;
    part[wv][1] = lc;
  }
  __syncthreads();
  __shared__ int last;
  if (threadIdx.x == 0) {
    double d = 0.0, cs = 0.0;
    for (int w = 0; w < FUSED_RAYS; ++w) {
      d += part[w][0];
      cs += part[w][1];
    }
    c.loss_part[2 * blockIdx.x] = d;
    c.loss_part[2 * blockIdx.x + 1] = cs;
    __threadfence();  // the partials are visible device-wide before the count says so
    last = atomicAdd(c.loss_count, 1u) == nb - 1;
  }
  __syncthreads();
  if (!last) return;
  __threadfence();
  // the last workgroup: every partial in block order (thread t: blocks t, t + 64 * FUSED_RAYS,
  // ...), then the wave butterfly and the waves in order -- one association for any timing
  double d = 0.0, cs = 0.0;
  for (unsigned b = threadIdx.x; b < nb; b += 64 * FUSED_RAYS) {
    d += c.loss_part[2 * b];
    cs += c.loss_part[2 * b + 1];
  }
  d = wsum_d(d);
  cs = wsum_d(cs);
  __syncthreads();  // part[][] is reused
  if (lane == 0) {
    part[wv][0] = d;
    part[wv][1] = cs;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double ds = 0.0, css = 0.0;
    for (int w = 0; w < FUSED_RAYS; ++w) {
      ds += part[w][0];
      css += part[w][1];
    }
    *c.loss_out = col_term ? ds + (double)(c.w_color * (float)css) : ds;
  }
}

int64_t fused_loss_blocks(int64_t N) { return (N + FUSED_RAYS - 1) / FUSED_RAYS; }

__device__ __forceinline__ void ray_grads_body(const RayCtx& c, int64_t block) {
  const int lane = threadIdx.x & 63;
  const int64_t r = block * RAY_WAVES + (threadIdx.x >> 6);
  if (r >= c.N) return;
  const bool act = lane < c.S && ray_ok(c, r);  // a dropped ray's gradients are 0
  const int64_t p = r * c.S + (lane < c.S ? lane : 0);
  // every job's point gradient and the depth loaded unconditionally (clamped), then summed
  // in job order and selected: no load waits alone in a branch
  double g[MAX_JOBS][3];
#pragma unroll
  for (int j = 0; j < MAX_JOBS; ++j) {
    const int jj = j < c.n_jobs ? j : 0;
#pragma unroll
    for (int k = 0; k < 3; ++k) g[j][k] = c.dpts[((int64_t)jj * c.P + p) * 3 + k];
  }
  const double zl = c.z[p];
  double dp[3] = {0.0, 0.0, 0.0};
#pragma unroll
  for (int j = 0; j < MAX_JOBS; ++j) {
#pragma unroll
    for (int k = 0; k < 3; ++k) dp[k] = j < c.n_jobs ? dp[k] + g[j][k] : dp[k];
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) dp[k] = act ? dp[k] : 0.0;
  const double z = act ? zl : 0.0;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const double go = wsum_d(dp[k]);
    const double gd = wsum_d(dp[k] * z);
    if (lane == 0) {
      if (c.g_rays_o) c.g_rays_o[r * 3 + k] = (float)go;
      if (c.g_rays_d) {
        float v = (float)gd;
        if (c.density && c.gnorm) {  // + d ||rays_d|| / d rays_d (torch.norm backward, 0 at norm 0)
          const float* d = c.rays_d + r * 3;
          const float n = sqrtf(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
          v = v + (n > 0.f ? c.gnorm[r] * (d[k] / n) : 0.f);
        }
        c.g_rays_d[r * 3 + k] = v;
      }
    }
  }
}

__global__ void __launch_bounds__(256) k_ray_grads(const RayCtx c) { ray_grads_body(c, blockIdx.x); }

// thread = (float4 column of the parameter vector, part): part p sums slab rows
// p, p+8, ... (independent loads in flight), the 8 partial sums meet in LDS.
constexpr int PR_COLS = 32, PR_PARTS = 8;
#ifndef NC_PR_AHEAD
#define NC_PR_AHEAD 4
#endif
constexpr int PR_AHEAD = NC_PR_AHEAD;  // slab rows in flight per thread (8 / 12: no gain, profiles/r04/ray_loads/ab_pr.log)
static_assert(PR_COLS * PR_PARTS == 64 * RAY_WAVES, "k_param_ray_reduce: one block size for both roles");
__device__ __forceinline__ void param_reduce_body(const ParamReduceCtx& c, int bx, int j) {
  // the per-workgroup partials are summed in float64 (rounded once at the end): bias
  // gradients cancel heavily across workgroups (k_mlp_dw's float64 bias sums)
  __shared__ double part[PR_PARTS][PR_COLS][4];
  // constant-index selects (dynamic indexing of the argument block spills it)
  const Job job = j == 0 ? c.jobs[0] : (j == 1 ? c.jobs[1] : c.jobs[2]);
  float* grad = j == 0 ? c.grad[0] : (j == 1 ? c.grad[1] : c.grad[2]);
  const int64_t np = j == 0 ? c.nparam[0] : (j == 1 ? c.nparam[1] : c.nparam[2]);
  if (!job.need_dw || grad == nullptr) return;
  const int col = threadIdx.x % PR_COLS, prt = threadIdx.x / PR_COLS;
  const int64_t e = ((int64_t)bx * PR_COLS + col) * 4;  // first parameter of the column
  if ((int64_t)bx * PR_COLS * 4 >= np) return;          // whole workgroup past the end
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  if (e < c.slab_stride) {  // slab rows are padded to slab_stride (multiple of 64 floats)
    const int w0 = j == 0 ? c.wg_off[0] : (j == 1 ? c.wg_off[1] : c.wg_off[2]);
    const int w1 = j == 0 ? c.wg_off[1] : (j == 1 ? c.wg_off[2] : c.wg_off[3]);
    const float* src = c.slab + (int64_t)w0 * c.slab_stride + e;
    auto row = [&](int w) { return *reinterpret_cast<const float4*>(src + (int64_t)w * c.slab_stride); };
    const int nw = w1 - w0;
    int w = prt;
    // PR_AHEAD rows in flight, added in the same order as one at a time (bit-identical sums)
    for (; w + (PR_AHEAD - 1) * PR_PARTS < nw; w += PR_AHEAD * PR_PARTS) {
      float4 v[PR_AHEAD];
#pragma unroll
      for (int u = 0; u < PR_AHEAD; ++u) v[u] = row(w + u * PR_PARTS);
#pragma unroll
      for (int u = 0; u < PR_AHEAD; ++u) {
        acc[0] += v[u].x; acc[1] += v[u].y; acc[2] += v[u].z; acc[3] += v[u].w;
      }
    }
    for (; w < nw; w += PR_PARTS) {
      const float4 v = row(w);
      acc[0] += v.x; acc[1] += v.y; acc[2] += v.z; acc[3] += v.w;
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) part[prt][col][k] = acc[k];
  __syncthreads();
  if (prt == 0) {
    double sv[4] = {part[0][col][0], part[0][col][1], part[0][col][2], part[0][col][3]};
#pragma unroll
    for (int q = 1; q < PR_PARTS; ++q)
#pragma unroll
      for (int k = 0; k < 4; ++k) sv[k] += part[q][col][k];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (e + k < np) grad[e + k] = (float)sv[k];
  }
}

__global__ void __launch_bounds__(PR_COLS * PR_PARTS) k_param_reduce(const ParamReduceCtx c) {
  param_reduce_body(c, blockIdx.x, blockIdx.y);
}

// the backward's last two steps in one launch: blocks [0, pr_blocks) sum the weight-
// gradient slabs (job = b / pr_x), the rest form d rays_o / d rays_d
__global__ void __launch_bounds__(PR_COLS * PR_PARTS) k_param_ray_reduce(const ParamReduceCtx pc, const RayCtx rc,
                                                                        int pr_x, int pr_blocks) {
  const int b = blockIdx.x;
  if (b < pr_blocks) param_reduce_body(pc, b % pr_x, b / pr_x);
  else ray_grads_body(rc, b - pr_blocks);
}

// ---- NICE.forward on caller points (decoder.py:336-370) ----
__global__ void k_points_assemble(const MlpCtx m, int stage, float* raw) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= m.P) return;
  float o[4] = {0.f, 0.f, 0.f, 0.f};
  if (stage == NC_STAGE_COLOR) {
    o[0] = m.rgb[p * 3 + 0];
    o[1] = m.rgb[p * 3 + 1];
    o[2] = m.rgb[p * 3 + 2];
  }
  if (stage == NC_STAGE_FINE || stage == NC_STAGE_COLOR) o[3] = m.occ[p] + m.occ[m.P + p];  // fine + middle
  else o[3] = m.occ[p];
#pragma unroll
  for (int k = 0; k < 4; ++k) raw[p * 4 + k] = o[k];
}

__global__ void k_points_split_grad(const MlpCtx m, int stage, const float* g_raw, float* gocc, float* grgb) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= m.P) return;
  gocc[p] = g_raw[p * 4 + 3];
  if (stage == NC_STAGE_COLOR) {
#pragma unroll
    for (int k = 0; k < 3; ++k) grgb[p * 3 + k] = g_raw[p * 4 + k];
  }
}

__global__ void k_points_grads(const MlpCtx m, double* g_pts) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= m.P) return;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    double s = 0.0;
    for (int j = 0; j < m.n_jobs; ++j) s += m.dpts[((int64_t)j * m.P + p) * 3 + k];
    g_pts[p * 3 + k] = s;
  }
}

// ---- launch wrappers ----
static inline unsigned ray_blocks(int64_t n) { return (unsigned)((n + RAY_WAVES - 1) / RAY_WAVES); }

int launch_depth_max(const float* gt, const uint8_t* valid, int64_t n, float* out, hipStream_t s) {
  hipLaunchKernelGGL(k_depth_max, dim3(1), dim3(1024), 0, s, gt, valid, n, out);
  return (int)hipGetLastError();
}
int launch_ray_setup(const RayCtx& c, const WImgCtx& wi, hipStream_t s) {
  hipLaunchKernelGGL(k_ray_setup, dim3(ray_blocks(c.N) + ray_fill_wgs(c) + (unsigned)(wi.n_jobs * wi.wgs_per_job)),
                     dim3(256), 0, s, c, wi);
  return (int)hipGetLastError();
}
int launch_composite_fwd(const RayCtx& c, hipStream_t s) {
  hipLaunchKernelGGL(k_composite_fwd, dim3(ray_blocks(c.N)), dim3(256), 0, s, c);
  return (int)hipGetLastError();
}
int launch_composite_fwd_loss(const RayCtx& c, hipStream_t s) {
  const unsigned nb = (unsigned)((c.N + FUSED_RAYS - 1) / FUSED_RAYS);
  hipLaunchKernelGGL(k_composite_fwd_loss, dim3(nb + (c.zero_fill && c.zero_n4 > c.zero_lo4 ? (unsigned)c.zero_wgs : 0u)),
                     dim3(64 * FUSED_RAYS), 0,
                     s, c);
  return (int)hipGetLastError();
}
int launch_composite_bwd(const RayCtx& c, hipStream_t s) {
  hipLaunchKernelGGL(k_composite_bwd, dim3(ray_blocks(c.N)), dim3(256), 0, s, c);
  return (int)hipGetLastError();
}
int launch_loss(const RayCtx& c, hipStream_t s) {
  hipLaunchKernelGGL(k_loss, dim3(1), dim3(LOSS_THREADS), 0, s, c);
  return (int)hipGetLastError();
}
int launch_ray_grads(const RayCtx& c, hipStream_t s) {
  hipLaunchKernelGGL(k_ray_grads, dim3(ray_blocks(c.N)), dim3(256), 0, s, c);
  return (int)hipGetLastError();
}
int launch_param_reduce(const ParamReduceCtx& c, int64_t max_nparam, hipStream_t s) {
  dim3 grid((unsigned)((max_nparam + 4 * PR_COLS - 1) / (4 * PR_COLS)), c.n_jobs);
  hipLaunchKernelGGL(k_param_reduce, grid, dim3(PR_COLS * PR_PARTS), 0, s, c);
  return (int)hipGetLastError();
}
int launch_param_ray_reduce(const ParamReduceCtx& c, int64_t max_nparam, const RayCtx& rc, hipStream_t s) {
  const int pr_x = (int)((max_nparam + 4 * PR_COLS - 1) / (4 * PR_COLS));
  const int pr_blocks = pr_x * c.n_jobs;
  hipLaunchKernelGGL(k_param_ray_reduce, dim3((unsigned)(pr_blocks + ray_blocks(rc.N))), dim3(PR_COLS * PR_PARTS), 0,
                     s, c, rc, pr_x, pr_blocks);
  return (int)hipGetLastError();
}
int launch_points_assemble(const MlpCtx& m, int stage, float* raw, hipStream_t s) {
  hipLaunchKernelGGL(k_points_assemble, dim3((unsigned)((m.P + 255) / 256)), dim3(256), 0, s, m, stage, raw);
  return (int)hipGetLastError();
}
int launch_points_split_grad(const MlpCtx& m, int stage, const float* g_raw, float* gocc, float* grgb,
                             hipStream_t s) {
  hipLaunchKernelGGL(k_points_split_grad, dim3((unsigned)((m.P + 255) / 256)), dim3(256), 0, s, m, stage,
                     g_raw, gocc, grgb);
  return (int)hipGetLastError();
}
int launch_points_prep(const MlpCtx& m, const WImgCtx& wi, float4* xyz, float4* pf, hipStream_t s) {
  hipLaunchKernelGGL(k_points_prep, dim3((unsigned)((m.P + 255) / 256) + (unsigned)(wi.n_jobs * wi.wgs_per_job)), dim3(256), 0,
                     s, m, wi, xyz, pf);
  return (int)hipGetLastError();
}
int launch_points_grads(const MlpCtx& m, double* g_pts, hipStream_t s) {
  hipLaunchKernelGGL(k_points_grads, dim3((unsigned)((m.P + 255) / 256)), dim3(256), 0, s, m, g_pts);
  return (int)hipGetLastError();
}

}  // namespace nc
