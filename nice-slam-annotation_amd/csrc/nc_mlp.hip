// nc_mlp.hip — point-batched NICE decoders on gfx950 (forward and backward).
//
// Restates, per sample point:
//   MLP.sample_grid_feature + F.grid_sample  decoder.py:179-188, common.py:280-295
//   GaussianFourierFeatureTransform          decoder.py:26-30
//   MLP.forward                              decoder.py:190-219
//   MLP_no_xyz.forward                       decoder.py:285-297
// and the autograd backward of all of it (weights, biases, Fourier B, grid
// features, point coordinates).
//
// Work decomposition: one launch per pass, gridDim.y = the stage's decoders
// (jobs), each workgroup keeps ONE decoder's weights resident in LDS and walks
// point chunks persistently.  Each wavefront owns 16 points in the "C layout"
// (nc_device.h) and runs every nn.Linear as v_mfma_f32_16x16x4_f32 chains
// (weights = A operand from LDS, activations = B operand straight from the
// previous layer's accumulators).
//
// Backward (per 64-point sub-chunk of a 4-wave workgroup):
//   * per wave: recompute the forward, then dX = W^T dZ chains (MFMA), the
//     Fourier chain, the trilinear scatter (float atomics) and point gradients;
//   * per layer: the four waves stage dZ / dF and the layer input through LDS
//     ([point][feature] images) and the weight gradient dW = dZ^T X is formed
//     by MFMAs that reduce over the 64 points; tiles are owned by waves and
//     accumulated in registers across all sub-chunks of the workgroup, then
//     flushed once into an LDS image of the flat parameter vector and written
//     to a per-workgroup slab (reduced by nc_rays.hip:k_param_reduce).
#include "nc_device.h"
#include "nc_internal.h"

#ifdef NC_ABL_FAST_TRIG  // timing-only ablation: hardware sin/cos (wrong for large arguments)
#define NC_SIN __sinf
#define NC_COS __cosf
#else
#define NC_SIN sinf
#define NC_COS cosf
#endif

namespace nc {

// ---------------------------------------------------------------------------
// weights: nn.Parameter storage -> LDS image (layout: Net<KIND>)
// ---------------------------------------------------------------------------
template <int KIND>
__device__ __forceinline__ void load_weights(float* lds, const nc_decoder_params& P) {
  using N = Net<KIND>;
  const int tid = threadIdx.x, nt = blockDim.x;
  for (int e = tid; e < N::WEIGHTS; e += nt) lds[e] = 0.f;
  __syncthreads();
#pragma unroll
  for (int L = 0; L < 5; ++L) {
    const int in = N::in_real(L), ld = N::lin_ld(L);
    float* dst = lds + N::lin_off(L);
    const float* W = P.lin_w[L];
    for (int e = tid; e < HID * in; e += nt) {
      const int o = e / in, c = e - o * in;
      dst[o * ld + N::pack_col(L, c)] = W[e];
    }
    for (int e = tid; e < HID; e += nt) lds[N::BL + L * HID + e] = P.lin_b[L][e];
  }
  if constexpr (N::XYZ) {
#pragma unroll
    for (int L = 0; L < 5; ++L) {
      const float* W = P.fc_w[L];
      float* dst = lds + N::WC + L * HID * N::LDC;
      for (int e = tid; e < HID * N::CD; e += nt) {
        const int o = e / N::CD, c = e - o * N::CD;
        dst[o * N::LDC + c] = W[e];
      }
      for (int e = tid; e < HID; e += nt) lds[N::BC + L * HID + e] = P.fc_b[L][e];
    }
    for (int e = tid; e < 3 * EMB; e += nt) {
      const int k = e / EMB, m = e - k * EMB;
      lds[N::FB + k * EMBP + m] = P.fourier_B[e];
    }
  }
  for (int e = tid; e < N::NOUT * HID; e += nt) lds[N::WO + e] = P.out_w[e];
  for (int e = tid; e < N::NOUT; e += nt) lds[N::BO + e] = P.out_b[e];
  __syncthreads();
}

// ---------------------------------------------------------------------------
// MFMA building blocks
// ---------------------------------------------------------------------------
// acc0/acc1 (output rows 0..15 / 16..31) += W[:, 16*qoff .. 16*(qoff+NQ)) * x
template <int NQ, int LD>
__device__ __forceinline__ void mm_fwd(const float* W, int qoff, const float* x, floatx4& a0,
                                       floatx4& a1, int i, int g) {
  const float* r0 = W + i * LD + 4 * g + 16 * qoff;
  const float* r1 = W + (16 + i) * LD + 4 * g + 16 * qoff;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const float4 w0 = *reinterpret_cast<const float4*>(r0 + 16 * q);
    const float4 w1 = *reinterpret_cast<const float4*>(r1 + 16 * q);
    a0 = mfma4(w0.x, x[4 * q + 0], a0);
    a1 = mfma4(w1.x, x[4 * q + 0], a1);
    a0 = mfma4(w0.y, x[4 * q + 1], a0);
    a1 = mfma4(w1.y, x[4 * q + 1], a1);
    a0 = mfma4(w0.z, x[4 * q + 2], a0);
    a1 = mfma4(w1.z, x[4 * q + 2], a1);
    a0 = mfma4(w0.w, x[4 * q + 3], a0);
    a1 = mfma4(w1.w, x[4 * q + 3], a1);
  }
}

// out[t] (input tiles ti0 .. ti0+NT) += W^T[16*(ti0+t) .., :] * dz   (dz: 32-wide C layout)
template <int NT, int LD>
__device__ __forceinline__ void mm_bwd(const float* W, int ti0, const float* dz, floatx4* out, int i,
                                       int g) {
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const float* row = W + feat_of(s, g) * LD + 16 * ti0 + i;
#pragma unroll
    for (int t = 0; t < NT; ++t) out[t] = mfma4(row[16 * t], dz[s], out[t]);
  }
}

__device__ __forceinline__ floatx4 bias4(const float* b, int g) {
  return floatx4{b[4 * g + 0], b[4 * g + 1], b[4 * g + 2], b[4 * g + 3]};
}

// ---------------------------------------------------------------------------
// Per-wave forward of one decoder for 16 points (recomputed in backward).
// ---------------------------------------------------------------------------
template <int KIND>
struct WaveRegs {
  float emb[Net<KIND>::XYZ ? 24 : 1];  // Fourier features, C layout over 96
  float c[Net<KIND>::CD / 4];          // grid features (fine: [fine | middle])
  float h[5][8];                       // block outputs h_0..h_4 (C layout)
  unsigned mask_lo, mask_hi;           // relu(Z) > 0 bits: layer L reg j -> bit 8L+j (L=4 in hi)
  float pf[3];                         // p.float()
  double p[3];                         // sample point (float64)
};

__device__ __forceinline__ bool mask_bit(unsigned lo, unsigned hi, int L, int j) {
  return L < 4 ? ((lo >> (8 * L + j)) & 1u) : ((hi >> j) & 1u);
}

template <int KIND>
__device__ __forceinline__ void wave_forward(const float* lds, const MlpCtx& ctx, int64_t p, bool valid,
                                             int i, int g, WaveRegs<KIND>& R, float out[4]) {
  using N = Net<KIND>;
  const nc_decoder_params& D = ctx.dec[KIND];
#pragma unroll
  for (int k = 0; k < 3; ++k) R.p[k] = valid ? ctx.pts[p * 3 + k] : D.bound[k][0];
  // grid features (decoder.py:179-188 / :196-202)
  float xyz[3];
  normalize_pt(R.p, D.bound, xyz);
  const nc_grid& G = ctx.grids[KIND];
  {
    Corners co;
    make_corners(G, xyz, co);
    if (grid_vec_ok(G)) gather8<true>(G, co, g, R.c);
    else gather8<false>(G, co, g, R.c);
  }
  if constexpr (KIND == K_FINE) {
    const nc_grid& GM = ctx.grids[K_MID];
    Corners cm;
    make_corners(GM, xyz, cm);
    if (grid_vec_ok(GM)) gather8<true>(GM, cm, g, R.c + 8);
    else gather8<false>(GM, cm, g, R.c + 8);
  }
  // Fourier embedding: sin(p.float() @ B), K=3 summed as fma(p2,B2, fma(p1,B1, p0*B0))
  // which is bit-identical to the CPU reference's sgemm for this shape.
  if constexpr (N::XYZ) {
#pragma unroll
    for (int k = 0; k < 3; ++k) R.pf[k] = (float)R.p[k];
    const float* B = lds + N::FB;
#pragma unroll
    for (int j = 0; j < 24; ++j) {
      const int m = feat_of(j, g);
      const float x = __builtin_fmaf(R.pf[2], B[2 * EMBP + m],
                                     __builtin_fmaf(R.pf[1], B[EMBP + m], R.pf[0] * B[m]));
      R.emb[j] = (m < EMB) ? NC_SIN(x) : 0.f;
    }
  }
  R.mask_lo = 0;
  R.mask_hi = 0;
#pragma unroll
  for (int L = 0; L < 5; ++L) {
    const float* bl = lds + N::BL + L * HID;
    floatx4 z0 = bias4(bl, g), z1 = bias4(bl + 16, g);
    const float* W = lds + N::lin_off(L);
    if (L == 0) {
      if constexpr (N::XYZ) mm_fwd<6, N::LD0>(W, 0, R.emb, z0, z1, i, g);
      else mm_fwd<2, N::LD0>(W, 0, R.c, z0, z1, i, g);
    } else if (L == 3) {
      if constexpr (N::XYZ) {
        mm_fwd<6, N::LD3>(W, 0, R.emb, z0, z1, i, g);
        mm_fwd<2, N::LD3>(W, 6, R.h[2], z0, z1, i, g);
      } else {
        mm_fwd<2, N::LD3>(W, 0, R.c, z0, z1, i, g);
        mm_fwd<2, N::LD3>(W, 2, R.h[2], z0, z1, i, g);
      }
    } else {
      mm_fwd<2, N::LDH>(W, 0, R.h[L > 0 ? L - 1 : 0], z0, z1, i, g);
    }
    float hh[8];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      hh[r] = z0[r] > 0.f ? z0[r] : 0.f;
      hh[4 + r] = z1[r] > 0.f ? z1[r] : 0.f;
    }
    unsigned bits = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) bits |= (hh[j] > 0.f ? 1u : 0u) << j;
    if (L < 4) R.mask_lo |= bits << (8 * L);
    else R.mask_hi = bits;
    if constexpr (N::XYZ) {
      const float* bc = lds + N::BC + L * HID;
      floatx4 f0, f1;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        f0[r] = hh[r] + bc[4 * g + r];
        f1[r] = hh[4 + r] + bc[16 + 4 * g + r];
      }
      mm_fwd<N::CD / 16, N::LDC>(lds + N::WC + L * HID * N::LDC, 0, R.c, f0, f1, i, g);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        R.h[L][r] = f0[r];
        R.h[L][4 + r] = f1[r];
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) R.h[L][j] = hh[j];
    }
  }
  // output_linear (VALU dot over the point's four lanes)
#pragma unroll
  for (int o = 0; o < 4; ++o) {
    if (o >= (KIND == K_COLOR ? 3 : 1)) { out[o] = 0.f; continue; }
    const float* wo = lds + N::WO + o * HID;
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) s = s + wo[feat_of(j, g)] * R.h[4][j];
    out[o] = sum_groups(s) + lds[N::BO + o];
  }
}

// Constant-index select: a dynamic index into the by-value kernel-argument block
// would make the compiler copy the whole block to scratch.
__device__ __forceinline__ Job pick_job(const Job (&jobs)[MAX_JOBS], unsigned y) {
  return y == 0 ? jobs[0] : (y == 1 ? jobs[1] : jobs[2]);
}

// ---------------------------------------------------------------------------
// forward kernel
// ---------------------------------------------------------------------------
template <int KIND>
__device__ __forceinline__ void fwd_job(const MlpCtx& ctx, const Job& job, float* lds) {
  load_weights<KIND>(lds, ctx.dec[KIND]);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
  const int waves = blockDim.x >> 6;
  const int64_t per = 16 * waves;
  const int64_t nblk = (ctx.P + per - 1) / per;
  for (int64_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
    // keep the (loop-invariant) LDS weight reads inside the loop: hoisting all of
    // them out of the persistent loop would need thousands of registers
    asm volatile("" ::: "memory");
    const int64_t p = blk * per + wave * 16 + i;
    const bool valid = p < ctx.P;
    WaveRegs<KIND> R;
    float out[4];
    wave_forward<KIND>(lds, ctx, p, valid, i, g, R, out);
    if (valid && g == 0) {
      if constexpr (KIND == K_COLOR) {
        ctx.rgb[p * 3 + 0] = out[0];
        ctx.rgb[p * 3 + 1] = out[1];
        ctx.rgb[p * 3 + 2] = out[2];
      } else {
        ctx.occ[(int64_t)job.slot * ctx.P + p] = out[0];
      }
    }
  }
}

__global__ void __launch_bounds__(FWD_THREADS) k_mlp_fwd(const MlpCtx ctx) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const Job job = pick_job(ctx.jobs, blockIdx.y);
  switch (job.kind) {
    case K_COARSE: fwd_job<K_COARSE>(ctx, job, lds); break;
    case K_MID: fwd_job<K_MID>(ctx, job, lds); break;
    case K_FINE: fwd_job<K_FINE>(ctx, job, lds); break;
    default: fwd_job<K_COLOR>(ctx, job, lds); break;
  }
}

// ---------------------------------------------------------------------------
// backward: weight-gradient phases
// ---------------------------------------------------------------------------
constexpr int CH = 64;  // points per sub-chunk (4 waves x 16)

// dW[16*to + r][16*ti + c] += sum over the 64 staged points of Y[pt][.] X[pt][.]
// Tiles tau = wave + 4*s (s < NS) of an NR x NC tile grid.  With BIAS, the owner
// of a first-column tile also adds the row sums of Y (the bias gradient) into the
// LDS accumulator bacc[16*to + r].
template <int NR, int NC, int NS, bool BIAS>
__device__ __forceinline__ void dw_phase(const float* Y, int ldY, const float* X, int ldX, floatx4* acc,
                                         float* bacc, int wave, int i, int g) {
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int tau = wave + 4 * s;
    if (tau < NR * NC) {
      const int to = tau / NC, ti = tau - to * NC;
      const float* y = Y + g * ldY + 16 * to + i;
      const float* x = X + g * ldX + 16 * ti + i;
      floatx4 a = acc[s];
      float bs = 0.f;
#pragma unroll
      for (int q = 0; q < CH / 4; ++q) {
        const float av = y[4 * q * ldY];
        a = mfma4(av, x[4 * q * ldX], a);
        if (BIAS) bs += av;
      }
      acc[s] = a;
      if (BIAS && ti == 0) {
        bs = sum_groups(bs);
        if (g == 0) atomicAdd(bacc + 16 * to + i, bs);
      }
    }
  }
}

// write 16 points x (4*NT) features of this wave (C layout) as rows of an LDS image
template <int NT>
__device__ __forceinline__ void stage_rows(float* img, int ld, int col0, const float* v, int row, int g) {
#pragma unroll
  for (int t = 0; t < NT; ++t)
    *reinterpret_cast<float4*>(img + row * ld + col0 + 16 * t + 4 * g) =
        float4{v[4 * t + 0], v[4 * t + 1], v[4 * t + 2], v[4 * t + 3]};
}

// flat-parameter index of a dW tile element, or -1 (padding)
template <int KIND>
struct PhaseMap {
  using N = Net<KIND>;
  // phase ids: 0 = out, 1..5 = pts_linears[4..0], 6..10 = fc_c[4..0], 11 = Fourier B
  __device__ static int64_t w_index(int ph, int row, int col) {
    if (ph == 0) return (row < N::NOUT) ? N::P_OUT_W + row * HID + col : -1;
    if (ph <= 5) {
      const int L = 5 - ph;
      const int rc = N::real_col(L, col);
      return rc < 0 ? -1 : N::p_lin_w(L) + (int64_t)row * N::in_real(L) + rc;
    }
    if (ph <= 10) {
      const int L = 10 - ph;
      return N::p_fc_w(L) + (int64_t)row * N::CD + col;
    }
    return (row < EMB && col < 3) ? N::P_B + (int64_t)col * EMB + row : -1;
  }
  __device__ static int64_t b_index(int ph, int row) {
    if (ph == 0) return row < N::NOUT ? N::P_OUT_B + row : -1;
    if (ph <= 5) return N::p_lin_b(5 - ph) + row;
    if (ph <= 10) return N::p_fc_b(10 - ph) + row;
    return -1;
  }
};

template <int KIND, int NR, int NC, int NS>
__device__ __forceinline__ void flush_phase(float* img, int ph, const floatx4* acc, int wave, int i, int g) {
  using PM = PhaseMap<KIND>;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int tau = wave + 4 * s;
    if (tau < NR * NC) {
      const int to = tau / NC, ti = tau - to * NC;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t idx = PM::w_index(ph, 16 * to + 4 * g + r, 16 * ti + i);
        if (idx >= 0) atomicAdd(img + idx, acc[s][r]);
      }
    }
  }
}

// slot bookkeeping per decoder kind
template <int KIND>
struct Slots {
  using N = Net<KIND>;
  static constexpr int NC0 = N::IN0 / 16, NC3 = N::IN3 / 16, NCC = N::CD / 16;
  static constexpr int ns(int tiles) { return (tiles + 3) / 4; }
  static constexpr int OUT = 0;
  static constexpr int L4 = OUT + ns(2);
  static constexpr int C4 = L4 + ns(4);
  static constexpr int L3 = C4 + (N::XYZ ? ns(2 * NCC) : 0);
  static constexpr int C3 = L3 + ns(2 * NC3);
  static constexpr int L2 = C3 + (N::XYZ ? ns(2 * NCC) : 0);
  static constexpr int C2 = L2 + ns(4);
  static constexpr int L1 = C2 + (N::XYZ ? ns(2 * NCC) : 0);
  static constexpr int C1 = L1 + ns(4);
  static constexpr int L0 = C1 + (N::XYZ ? ns(2 * NCC) : 0);
  static constexpr int C0 = L0 + ns(2 * NC0);
  static constexpr int FB = C0 + (N::XYZ ? ns(2 * NCC) : 0);
  static constexpr int TOTAL = FB + (N::XYZ ? ns(6) : 0);
  __host__ __device__ static constexpr int lin(int L) {
    return L == 4 ? L4 : L == 3 ? L3 : L == 2 ? L2 : L == 1 ? L1 : L0;
  }
  __host__ __device__ static constexpr int fc(int L) {
    return L == 4 ? C4 : L == 3 ? C3 : L == 2 ? C2 : L == 1 ? C1 : C0;
  }
};

// LDS carve-up of the backward kernel (floats)
template <int KIND>
struct BwdLds {
  using N = Net<KIND>;
  static constexpr int LDCB = N::CD + 16;  // c image leading dim (== 16 mod 32)
  static constexpr int CBUF = N::WEIGHTS;
  static constexpr int STAGE = CBUF + (N::XYZ ? CH * LDCB : 0);
  static constexpr int STAGE_FLOATS = CH * (48 + 144);
  static constexpr int BACC = STAGE + STAGE_FLOATS;  // bias-gradient accumulators
  // per phase id (see PhaseMap): 0 out (16), 1..5 pts_linears[4..0] (32 each), 6..10 fc_c[4..0]
  __host__ __device__ static constexpr int bacc_off(int ph) { return ph == 0 ? 0 : 16 + 32 * (ph - 1); }
  static constexpr int BACC_FLOATS = 16 + 32 * 10;
  static constexpr int TOTAL = BACC + BACC_FLOATS;
};

__host__ __device__ constexpr int cmax(int a, int b) { return a > b ? a : b; }
constexpr int BWD_LDS_FLOATS =
    cmax(cmax(BwdLds<K_COARSE>::TOTAL, BwdLds<K_MID>::TOTAL), cmax(BwdLds<K_FINE>::TOTAL, BwdLds<K_COLOR>::TOTAL));
constexpr int FWD_LDS_FLOATS =
    cmax(cmax(Net<K_COARSE>::WEIGHTS, Net<K_MID>::WEIGHTS), cmax(Net<K_FINE>::WEIGHTS, Net<K_COLOR>::WEIGHTS));
static_assert(BWD_LDS_FLOATS * 4 <= 160 * 1024, "backward LDS budget");

template <int KIND>
__device__ __forceinline__ void bwd_job(const MlpCtx& ctx, const Job& job, float* lds) {
  using N = Net<KIND>;
  using SL = Slots<KIND>;
  using BL = BwdLds<KIND>;
  load_weights<KIND>(lds, ctx.dec[KIND]);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
  const int row = wave * 16 + i;
  float* cbuf = lds + BL::CBUF;
  float* stg = lds + BL::STAGE;
  const bool need_dw = job.need_dw != 0;
  const bool need_grid = job.need_grid != 0 && ctx.grids[KIND].grad != nullptr;
  const bool need_coord = job.need_coord != 0;
  const bool need_dc = need_grid || need_coord;

  floatx4 acc[SL::TOTAL];
#pragma unroll
  for (int s = 0; s < SL::TOTAL; ++s) acc[s] = zero4();
  float* bacc = lds + BL::BACC;
  for (int e = threadIdx.x; e < BL::BACC_FLOATS; e += blockDim.x) bacc[e] = 0.f;
  __syncthreads();

  const int64_t nblk = (ctx.P + CH - 1) / CH;
  for (int64_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
    asm volatile("" ::: "memory");  // no hoisting of LDS weight reads (see fwd_job)
    const int64_t p = blk * CH + row;
    const bool valid = p < ctx.P;
    WaveRegs<KIND> R;
    float out[4];
    wave_forward<KIND>(lds, ctx, p, valid, i, g, R, out);

    // upstream gradient of this decoder's output (decoder.py:345-370 stage wiring)
    float dout[4] = {0.f, 0.f, 0.f, 0.f};
    if (valid) {
      if constexpr (KIND == K_COLOR) {
        dout[0] = ctx.grgb[p * 3 + 0];
        dout[1] = ctx.grgb[p * 3 + 1];
        dout[2] = ctx.grgb[p * 3 + 2];
      } else {
        dout[0] = ctx.gocc[p];
      }
    }
    float dh[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float s = 0.f;
#pragma unroll
      for (int o = 0; o < N::NOUT; ++o) s = s + lds[N::WO + o * HID + feat_of(j, g)] * dout[o];
      dh[j] = s;
    }
    if (need_dw) {
      float* Y = stg;
      float* X = stg + CH * 16;
      *reinterpret_cast<float4*>(Y + row * 16 + 4 * g) =
          g == 0 ? float4{dout[0], dout[1], dout[2], dout[3]} : float4{0.f, 0.f, 0.f, 0.f};
      stage_rows<2>(X, 48, 0, R.h[4], row, g);
      if constexpr (N::XYZ) stage_rows<N::CD / 16>(cbuf, BL::LDCB, 0, R.c, row, g);
      __syncthreads();
      dw_phase<1, 2, 1, true>(Y, 16, X, 48, acc + SL::OUT, bacc + BL::bacc_off(0), wave, i, g);
      __syncthreads();
    }

    floatx4 dc[2] = {zero4(), zero4()};
    floatx4 demb[6] = {zero4(), zero4(), zero4(), zero4(), zero4(), zero4()};
#pragma unroll
    for (int L = 4; L >= 0; --L) {
      float dz[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) dz[j] = mask_bit(R.mask_lo, R.mask_hi, L, j) ? dh[j] : 0.f;
      // dF (fc_c branch) -> d features (only the decoder's own 32 channels carry grad)
      if constexpr (N::XYZ) {
        if (need_dc) mm_bwd<2, N::LDC>(lds + N::WC + L * HID * N::LDC, 0, dh, dc, i, g);
      }
      // weight-gradient phases for this block (before dh is overwritten)
      if (need_dw) {
        float* Y = stg;
        float* X = stg + CH * 48;
        stage_rows<2>(Y, 48, 0, dz, row, g);
        int ldx;
        if (L == 0) {
          if constexpr (N::XYZ) { ldx = 112; stage_rows<6>(X, ldx, 0, R.emb, row, g); }
          else { ldx = 48; stage_rows<2>(X, ldx, 0, R.c, row, g); }
        } else if (L == 3) {
          if constexpr (N::XYZ) {
            ldx = 144;
            stage_rows<6>(X, ldx, 0, R.emb, row, g);
            stage_rows<2>(X, ldx, 96, R.h[2], row, g);
          } else {
            ldx = 80;
            stage_rows<2>(X, ldx, 0, R.c, row, g);
            stage_rows<2>(X, ldx, 32, R.h[2], row, g);
          }
        } else {
          ldx = 48;
          stage_rows<2>(X, ldx, 0, R.h[L > 0 ? L - 1 : 0], row, g);
        }
        __syncthreads();
        if (L == 0) {
          dw_phase<2, SL::NC0, SL::ns(2 * SL::NC0), true>(Y, 48, X, ldx, acc + SL::L0, bacc + BL::bacc_off(5 - L), wave, i, g);
        } else if (L == 3) {
          dw_phase<2, SL::NC3, SL::ns(2 * SL::NC3), true>(Y, 48, X, ldx, acc + SL::L3, bacc + BL::bacc_off(5 - L), wave, i, g);
        } else {
          dw_phase<2, 2, 1, true>(Y, 48, X, ldx, acc + SL::lin(L), bacc + BL::bacc_off(5 - L), wave, i, g);
        }
        __syncthreads();
        if constexpr (N::XYZ) {
          stage_rows<2>(Y, 48, 0, dh, row, g);
          __syncthreads();
          dw_phase<2, SL::NCC, SL::ns(2 * SL::NCC), true>(Y, 48, cbuf, BL::LDCB, acc + SL::fc(L),
                                                          bacc + BL::bacc_off(10 - L), wave, i, g);
          __syncthreads();
        }
      }
      // dX = W_L^T dZ
      const float* W = lds + N::lin_off(L);
      if (L == 0) {
        if constexpr (N::XYZ) mm_bwd<6, N::LD0>(W, 0, dz, demb, i, g);
        else if (need_dc) mm_bwd<2, N::LD0>(W, 0, dz, dc, i, g);
      } else if (L == 3) {
        floatx4 t2[2] = {zero4(), zero4()};
        if constexpr (N::XYZ) {
          mm_bwd<6, N::LD3>(W, 0, dz, demb, i, g);
          mm_bwd<2, N::LD3>(W, 6, dz, t2, i, g);
        } else {
          if (need_dc) mm_bwd<2, N::LD3>(W, 0, dz, dc, i, g);
          mm_bwd<2, N::LD3>(W, 2, dz, t2, i, g);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          dh[r] = t2[0][r];
          dh[4 + r] = t2[1][r];
        }
      } else {
        floatx4 t2[2] = {zero4(), zero4()};
        mm_bwd<2, N::LDH>(W, 0, dz, t2, i, g);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          dh[r] = t2[0][r];
          dh[4 + r] = t2[1][r];
        }
      }
    }

    // Fourier chain: d emb -> d x (cos), -> d p.float() and d B
    float dpf[3] = {0.f, 0.f, 0.f};
    if constexpr (N::XYZ) {
      const float* B = lds + N::FB;
      float dx[24];
#pragma unroll
      for (int j = 0; j < 24; ++j) {
        const int m = feat_of(j, g);
        const float x = __builtin_fmaf(R.pf[2], B[2 * EMBP + m],
                                       __builtin_fmaf(R.pf[1], B[EMBP + m], R.pf[0] * B[m]));
        dx[j] = (m < EMB) ? demb[j >> 2][j & 3] * NC_COS(x) : 0.f;
      }
      if (need_coord) {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          float s = 0.f;
#pragma unroll
          for (int j = 0; j < 24; ++j) s = s + B[k * EMBP + feat_of(j, g)] * dx[j];
          dpf[k] = sum_groups(s);
        }
      }
      if (need_dw) {
        float* Y = stg;
        float* X = stg + CH * 112;
        stage_rows<6>(Y, 112, 0, dx, row, g);
        *reinterpret_cast<float4*>(X + row * 16 + 4 * g) =
            g == 0 ? float4{R.pf[0], R.pf[1], R.pf[2], 0.f} : float4{0.f, 0.f, 0.f, 0.f};
        __syncthreads();
        dw_phase<6, 1, 2, false>(Y, 112, X, 16, acc + SL::FB, nullptr, wave, i, g);
        __syncthreads();
      }
    }

    // hand the trilinear backward to k_grid_bwd: d features (this decoder's own 32
    // channels, C layout) and the Fourier part of the point gradient
    if (need_dc && valid) {
      float* dst = ctx.dcbuf + ((int64_t)job.slot * ctx.P + p) * HID;
      *reinterpret_cast<float4*>(dst + 4 * g) = float4{dc[0][0], dc[0][1], dc[0][2], dc[0][3]};
      *reinterpret_cast<float4*>(dst + 16 + 4 * g) = float4{dc[1][0], dc[1][1], dc[1][2], dc[1][3]};
    }
    if (need_coord && valid && g == 0) {
      double* dst = ctx.dpts + ((int64_t)job.slot * ctx.P + p) * 3;
#pragma unroll
      for (int k = 0; k < 3; ++k) dst[k] = (double)dpf[k];
    }
  }

  if (!need_dw) return;
  // flush register-resident dW tiles -> LDS image of the flat parameter vector -> slab
  __syncthreads();
  float* img = lds;
  for (int e = threadIdx.x; e < N::NPARAM; e += blockDim.x) img[e] = 0.f;
  __syncthreads();
  flush_phase<KIND, 1, 2, 1>(img, 0, acc + SL::OUT, wave, i, g);
#pragma unroll
  for (int L = 4; L >= 0; --L) {
    if (L == 0) flush_phase<KIND, 2, SL::NC0, SL::ns(2 * SL::NC0)>(img, 5 - L, acc + SL::L0, wave, i, g);
    else if (L == 3) flush_phase<KIND, 2, SL::NC3, SL::ns(2 * SL::NC3)>(img, 5 - L, acc + SL::L3, wave, i, g);
    else flush_phase<KIND, 2, 2, 1>(img, 5 - L, acc + SL::lin(L), wave, i, g);
    if constexpr (N::XYZ)
      flush_phase<KIND, 2, SL::NCC, SL::ns(2 * SL::NCC)>(img, 10 - L, acc + SL::fc(L), wave, i, g);
  }
  if constexpr (N::XYZ) flush_phase<KIND, 6, 1, 2>(img, 11, acc + SL::FB, wave, i, g);
  // bias gradients from the LDS accumulators
  for (int e = threadIdx.x; e < BL::BACC_FLOATS; e += blockDim.x) {
    int ph, row;
    if (e < 16) { ph = 0; row = e; }
    else { ph = 1 + (e - 16) / 32; row = (e - 16) % 32; }
    if (ph > 5 && !N::XYZ) continue;
    const int64_t bi = PhaseMap<KIND>::b_index(ph, row);
    if (bi >= 0) img[bi] += bacc[e];
  }
  __syncthreads();
  float* slab = ctx.slab + ((int64_t)blockIdx.y * ctx.slab_wgs + blockIdx.x) * ctx.slab_stride;
  for (int e = threadIdx.x; e < N::NPARAM; e += blockDim.x) slab[e] = img[e];
}

__global__ void __launch_bounds__(BWD_THREADS) k_mlp_bwd(const MlpCtx ctx) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const Job job = pick_job(ctx.jobs, blockIdx.y);
  switch (job.kind) {
    case K_COARSE: bwd_job<K_COARSE>(ctx, job, lds); break;
    case K_MID: bwd_job<K_MID>(ctx, job, lds); break;
    case K_FINE: bwd_job<K_FINE>(ctx, job, lds); break;
    default: bwd_job<K_COLOR>(ctx, job, lds); break;
  }
}

// ---------------------------------------------------------------------------
// launch wrappers
// ---------------------------------------------------------------------------
int mlp_fwd_lds_bytes() { return FWD_LDS_FLOATS * 4; }
int mlp_bwd_lds_bytes() { return BWD_LDS_FLOATS * 4; }
int64_t max_param_count() {
  return cmax(cmax((int)Net<K_COARSE>::NPARAM, (int)Net<K_MID>::NPARAM),
              cmax((int)Net<K_FINE>::NPARAM, (int)Net<K_COLOR>::NPARAM));
}

int launch_mlp_fwd(const MlpCtx& c, int grid_x, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)k_mlp_fwd, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       mlp_fwd_lds_bytes());
    if (e != hipSuccess) return (int)e;
    attr = true;
  }
  dim3 grid(grid_x, c.n_jobs);
  hipLaunchKernelGGL(k_mlp_fwd, grid, dim3(FWD_THREADS), mlp_fwd_lds_bytes(), s, c);
  return (int)hipGetLastError();
}

int launch_mlp_bwd(const MlpCtx& c, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)k_mlp_bwd, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       mlp_bwd_lds_bytes());
    if (e != hipSuccess) return (int)e;
    attr = true;
  }
  dim3 grid(c.slab_wgs, c.n_jobs);
  hipLaunchKernelGGL(k_mlp_bwd, grid, dim3(BWD_THREADS), mlp_bwd_lds_bytes(), s, c);
  return (int)hipGetLastError();
}

}  // namespace nc
