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
#include "nc_grid.h"
#include "nc_internal.h"
#include "nc_wimage.h"

// A/B build: -DNC_MFMA_F32 runs the forward decoder GEMMs on the exact-f32 MFMA
// (v_mfma_f32_16x16x4_f32, the round-1 kernel) instead of split-f16.

namespace nc {

// ---------------------------------------------------------------------------
// weights: nn.Parameter storage -> LDS image (layout: Net<KIND>)
// Every thread first issues ALL of its global loads (one register array per
// parameter tensor, compile-time trip counts for the NT-thread workgroup), then
// zero-fills the padding of the image and stores: one memory round trip for the
// whole prologue instead of one per tensor.
// ---------------------------------------------------------------------------
template <int CNT, int NT>
struct SegRegs {
  static constexpr int PER = (CNT + NT - 1) / NT;
  float v[PER];
  __device__ __forceinline__ void load(const float* src) {
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int e = (int)threadIdx.x + k * NT;
      v[k] = (e < CNT) ? src[e] : 0.f;
    }
  }
  template <typename F>
  __device__ __forceinline__ void store(float* lds, F dst) const {
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int e = (int)threadIdx.x + k * NT;
      if (e < CNT) lds[dst(e)] = v[k];
    }
  }
};

template <int KIND, int PADW, int NT>
__device__ __forceinline__ void load_weights(float* lds, const nc_decoder_params& P) {
  using N = Net<KIND, PADW>;
  constexpr int CDW = N::XYZ ? HID * N::CD : 1, CB = N::XYZ ? HID : 1, NB = N::XYZ ? 3 * EMB : 1;
  SegRegs<HID * N::in_real(0), NT> w0;
  SegRegs<HID * N::in_real(1), NT> w1;
  SegRegs<HID * N::in_real(2), NT> w2;
  SegRegs<HID * N::in_real(3), NT> w3;
  SegRegs<HID * N::in_real(4), NT> w4;
  SegRegs<5 * HID, NT> bl;  // the five biases, gathered below
  SegRegs<CDW, NT> c0, c1, c2, c3, c4;
  SegRegs<5 * CB, NT> bc;
  SegRegs<NB, NT> fb;
  SegRegs<N::NOUT * HID + N::NOUT, NT> ow;
  w0.load(P.lin_w[0]); w1.load(P.lin_w[1]); w2.load(P.lin_w[2]); w3.load(P.lin_w[3]); w4.load(P.lin_w[4]);
#pragma unroll
  for (int k = 0; k < bl.PER; ++k) {  // 5 x 32 biases: tensor e / 32, entry e % 32
    const int e = (int)threadIdx.x + k * NT;
    const int L = e >> 5;
    const float* b = L == 0 ? P.lin_b[0] : L == 1 ? P.lin_b[1] : L == 2 ? P.lin_b[2] : L == 3 ? P.lin_b[3] : P.lin_b[4];
    bl.v[k] = (e < 5 * HID) ? b[e & 31] : 0.f;
  }
  if constexpr (N::XYZ) {
    c0.load(P.fc_w[0]); c1.load(P.fc_w[1]); c2.load(P.fc_w[2]); c3.load(P.fc_w[3]); c4.load(P.fc_w[4]);
#pragma unroll
    for (int k = 0; k < bc.PER; ++k) {
      const int e = (int)threadIdx.x + k * NT;
      const int L = e >> 5;
      const float* b = L == 0 ? P.fc_b[0] : L == 1 ? P.fc_b[1] : L == 2 ? P.fc_b[2] : L == 3 ? P.fc_b[3] : P.fc_b[4];
      bc.v[k] = (e < 5 * HID) ? b[e & 31] : 0.f;
    }
    fb.load(P.fourier_B);
  }
#pragma unroll
  for (int k = 0; k < ow.PER; ++k) {
    const int e = (int)threadIdx.x + k * NT;
    ow.v[k] = (e < N::NOUT * HID) ? P.out_w[e] : (e < N::NOUT * HID + N::NOUT ? P.out_b[e - N::NOUT * HID] : 0.f);
  }
  // zero the image (padding columns / rows stay 0) while the loads are in flight
  for (int e = threadIdx.x; e < N::WEIGHTS; e += NT) lds[e] = 0.f;
  __syncthreads();
  auto lin = [&](int L) {
    return [=](int e) {
      const int in = N::in_real(L);
      const int o = e / in, c = e - o * in;
      return N::lin_off(L) + o * N::lin_ld(L) + N::pack_col(L, c);
    };
  };
  w0.store(lds, lin(0)); w1.store(lds, lin(1)); w2.store(lds, lin(2)); w3.store(lds, lin(3)); w4.store(lds, lin(4));
  bl.store(lds, [](int e) { return N::BL + e; });
  if constexpr (N::XYZ) {
    auto fc = [&](int L) {
      return [=](int e) {
        const int o = e / N::CD, c = e - o * N::CD;
        return N::WC + L * HID * N::LDC + o * N::LDC + c;
      };
    };
    c0.store(lds, fc(0)); c1.store(lds, fc(1)); c2.store(lds, fc(2)); c3.store(lds, fc(3)); c4.store(lds, fc(4));
    bc.store(lds, [](int e) { return N::BC + e; });
    fb.store(lds, [](int e) {
      const int k = e / EMB, m = e - k * EMB;
      return N::FB + k * EMBP + m;
    });
  }
  ow.store(lds, [](int e) { return e < N::NOUT * HID ? N::WO + e : N::BO + (e - N::NOUT * HID); });
  __syncthreads();
}

// Split-f16 forward weight image (NetH, nc_device.h), prebuilt in global memory by the
// kernel before k_mlp_fwd (nc_wimage.h) and copied flat into LDS; its builders' range
// flags fold into amax (the max |w| of the split weights).
template <int KIND, int NT>
__device__ __forceinline__ void copy_wimage(char* lds, const char* img, float& amax) {
  using H = NetH<KIND>;
  const float4* src = reinterpret_cast<const float4*>(img);
  for (int e = threadIdx.x; e < H::BYTES / 16; e += NT) reinterpret_cast<float4*>(lds)[e] = src[e];
  const uint32_t* fl = reinterpret_cast<const uint32_t*>(img + H::BYTES);
  uint32_t f = 0u;
#pragma unroll
  for (int k = 0; k < WIMG_WGS; ++k) f |= fl[k];
  if (f) amax = __builtin_inff();
  __syncthreads();
}

// acc (output rows 16 ob + 4g + r) += M[:, block kb] x, both 16-row output blocks,
// T tiles sharing the weight fragments (forward image rows kb*32 + o; M3: the third planes):
// hh += Wh xh, mx += Wh xl + (Wm + W3) xh (units 2^-11)
template <int T>
__device__ __forceinline__ void mac_fwd(const char* M, const char* M3, int kb, const half8 (&xh)[T],
                                        const half8 (&xl)[T], floatx4 (&hh)[T][2], floatx4 (&mx)[T][2],
                                        int i, int g) {
#pragma unroll
  for (int ob = 0; ob < 2; ++ob) {
    const int r = kb * 32 + ob * 16 + i;
    const char* row = M + r * HROW;
    const half8 wh = *reinterpret_cast<const half8*>(row + hchunk(r, g, 0));
    const half8 wl = *reinterpret_cast<const half8*>(row + hchunk(r, g, 1));
#pragma unroll
    for (int t = 0; t < T; ++t) {
      hh[t][ob] = mfma16(wh, xh[t], hh[t][ob]);
      mx[t][ob] = mfma16(wh, xl[t], mx[t][ob]);
      mx[t][ob] = mfma16(wl, xh[t], mx[t][ob]);
    }
  }
  // the third planes after both blocks' main products (their fragments not live beside those)
#pragma unroll
  for (int ob = 0; ob < 2; ++ob) {
    const int r = kb * 32 + ob * 16 + i;
    const half8 w3 = *reinterpret_cast<const half8*>(M3 + r * HROW3 + hchunk3(r, g));
#pragma unroll
    for (int t = 0; t < T; ++t) mx[t][ob] = mfma16(w3, xh[t], mx[t][ob]);
  }
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
  // software-pipelined: step q+1's weight reads are issued before step q's MFMAs
  float4 w0 = *reinterpret_cast<const float4*>(r0);
  float4 w1 = *reinterpret_cast<const float4*>(r1);
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    float4 n0 = w0, n1 = w1;
    if (q + 1 < NQ) {
      n0 = *reinterpret_cast<const float4*>(r0 + 16 * (q + 1));
      n1 = *reinterpret_cast<const float4*>(r1 + 16 * (q + 1));
    }
    a0 = mfma4(w0.x, x[4 * q + 0], a0);
    a1 = mfma4(w1.x, x[4 * q + 0], a1);
    a0 = mfma4(w0.y, x[4 * q + 1], a0);
    a1 = mfma4(w1.y, x[4 * q + 1], a1);
    a0 = mfma4(w0.z, x[4 * q + 2], a0);
    a1 = mfma4(w1.z, x[4 * q + 2], a1);
    a0 = mfma4(w0.w, x[4 * q + 3], a0);
    a1 = mfma4(w1.w, x[4 * q + 3], a1);
    w0 = n0;
    w1 = n1;
  }
}

// T independent 16-point tiles through the same weights: 2T accumulation chains
// interleaved, so one tile's dependency bubbles are filled by the other's MFMAs.
template <int NQ, int LD, int T>
__device__ __forceinline__ void mm_fwd_t(const float* W, int qoff, const float* (&x)[T], floatx4 (&a0)[T],
                                         floatx4 (&a1)[T], int i, int g) {
  const float* r0 = W + i * LD + 4 * g + 16 * qoff;
  const float* r1 = W + (16 + i) * LD + 4 * g + 16 * qoff;
  float4 w0 = *reinterpret_cast<const float4*>(r0);
  float4 w1 = *reinterpret_cast<const float4*>(r1);
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    float4 n0 = w0, n1 = w1;
    if (q + 1 < NQ) {
      n0 = *reinterpret_cast<const float4*>(r0 + 16 * (q + 1));
      n1 = *reinterpret_cast<const float4*>(r1 + 16 * (q + 1));
    }
    const float wa[4] = {w0.x, w0.y, w0.z, w0.w}, wb[4] = {w1.x, w1.y, w1.z, w1.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
#pragma unroll
      for (int t = 0; t < T; ++t) {
        a0[t] = mfma4(wa[k], x[t][4 * q + k], a0[t]);
        a1[t] = mfma4(wb[k], x[t][4 * q + k], a1[t]);
      }
    }
    w0 = n0;
    w1 = n1;
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
// Per-point activation record saved by the forward for the backward kernels
// (float offsets; every block starts on a 16-byte boundary):
//   [h_0..h_4 5x32] [c CD] [relu masks: lane-group g -> u32 lo, hi] [p.float(), 0]
// The Fourier features are not stored: k_mlp_dw recomputes them from p.float()
// with the forward's own fourier_sin (bit-identical, ~110 MB less traffic a step).
// Backward record written by k_mlp_dx right after it (same point, offset LEN):
// [dh_0..dh_4 5x32] [dx 96 (xyz)] [d out, 0-padded to 4] where dh_L is
// d loss / d h_L (block L's output) and dx = d loss / d (p @ B).
// ---------------------------------------------------------------------------
template <int KIND>
struct Rec {
  using N = Net<KIND>;
  static constexpr int H = 0;
  static constexpr int C = H + 5 * HID;
  static constexpr int M = C + N::CD;
  static constexpr int PF = M + 8;           // p.float() (x, y, z, 0)
  static constexpr int LEN = PF + 4;
  static constexpr int DH = 0;
  static constexpr int DOUT = 5 * HID;       // d loss / d output (4; unused rows 0)
  static constexpr int DLEN = DOUT + 4;
  static constexpr int STRIDE = LEN + DLEN;  // one point: [forward record | backward record]
  static_assert(STRIDE % 32 == 16, "record stride must be 16 mod 32 (k_mlp_dw operand banks)");
};

template <int NT>
__device__ __forceinline__ void store_rows(float* dst, const float* v, int g) {
#pragma unroll
  for (int t = 0; t < NT; ++t)
    *reinterpret_cast<float4*>(dst + 16 * t + 4 * g) = float4{v[4 * t + 0], v[4 * t + 1], v[4 * t + 2], v[4 * t + 3]};
}


// ---------------------------------------------------------------------------
// Per-wave forward of one decoder for 16 points (recomputed in backward).
// ---------------------------------------------------------------------------
template <int KIND>
struct WaveRegs {
  float emb[Net<KIND>::XYZ ? 24 : 1];  // Fourier features, C layout over 96
  float c[Net<KIND>::CD / 4];          // grid features (fine: [fine | middle])
  float h[8];                          // current block output h_L (C layout); h_4 at the end
  float h2[8];                         // h_2, the skip input of block 3
  unsigned mask_lo, mask_hi;           // relu(Z) > 0 bits: layer L reg j -> bit 8L+j (L=4 in hi)
  float pf[3];                         // p.float()
};

__device__ __forceinline__ bool mask_bit(unsigned lo, unsigned hi, int L, int j) {
  return L < 4 ? ((lo >> (8 * L + j)) & 1u) : ((hi >> j) & 1u);
}

template <int KIND, int T>
__device__ __forceinline__ void wave_forward(const float* lds, int i, int g, WaveRegs<KIND> (&R)[T],
                                             float (&out)[T][4], float* const (&rec)[T], bool keep_h) {
  // R[t].pf / R[t].c: the tiles' inputs (grid features of decoder.py:179-188 /
  // :196-202, interpolated by k_grid_gather), loaded by the caller.  rec[t] != nullptr:
  // the point's activation record (Rec<KIND>) is written as each piece is produced.
  using N = Net<KIND, PADW_FWD>;
  // Fourier embedding: sin(p.float() @ B), K=3 summed as fma(p2,B2, fma(p1,B1, p0*B0))
  // which is bit-identical to the CPU reference's sgemm for this shape.
  if constexpr (N::XYZ) {
    const float* B = lds + N::FB;
#pragma unroll
    for (int j = 0; j < 24; ++j) {
      const int m = feat_of(j, g);
#pragma unroll
      for (int t = 0; t < T; ++t) {
        const float x = __builtin_fmaf(R[t].pf[2], B[2 * EMBP + m],
                                       __builtin_fmaf(R[t].pf[1], B[EMBP + m], R[t].pf[0] * B[m]));
        R[t].emb[j] = (m < EMB) ? fourier_sin(x) : 0.f;
      }
    }
  }
#pragma unroll
  for (int t = 0; t < T; ++t) R[t].mask_lo = R[t].mask_hi = 0;
  const float* xemb[T];
  const float* xc[T];
  const float* xh[T];
  const float* xh2[T];
#pragma unroll
  for (int t = 0; t < T; ++t) {
    xemb[t] = R[t].emb;
    xc[t] = R[t].c;
    xh[t] = R[t].h;
    xh2[t] = R[t].h2;
  }
#pragma unroll
  for (int L = 0; L < 5; ++L) {
    const float* bl = lds + N::BL + L * HID;
    floatx4 z0[T], z1[T];
#pragma unroll
    for (int t = 0; t < T; ++t) {
      z0[t] = bias4(bl, g);
      z1[t] = bias4(bl + 16, g);
    }
    const float* W = lds + N::lin_off(L);
    if (L == 0) {
      if constexpr (N::XYZ) mm_fwd_t<6, N::LD0, T>(W, 0, xemb, z0, z1, i, g);
      else mm_fwd_t<2, N::LD0, T>(W, 0, xc, z0, z1, i, g);
    } else if (L == 3) {
      if constexpr (N::XYZ) {
        mm_fwd_t<6, N::LD3, T>(W, 0, xemb, z0, z1, i, g);
        mm_fwd_t<2, N::LD3, T>(W, 6, xh2, z0, z1, i, g);
      } else {
        mm_fwd_t<2, N::LD3, T>(W, 0, xc, z0, z1, i, g);
        mm_fwd_t<2, N::LD3, T>(W, 2, xh2, z0, z1, i, g);
      }
    } else {
      mm_fwd_t<2, N::LDH, T>(W, 0, xh, z0, z1, i, g);
    }
    // relu and its mask from one compare per value (no IEEE-canonicalising max pair)
    floatx4 f0[T], f1[T];
    const float* bc = lds + N::BC + L * HID;
#pragma unroll
    for (int t = 0; t < T; ++t) {
      float hh[8];
      unsigned bits = 0;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bool p0 = z0[t][r] > 0.f, p1 = z1[t][r] > 0.f;
        hh[r] = p0 ? z0[t][r] : 0.f;
        hh[4 + r] = p1 ? z1[t][r] : 0.f;
        bits |= (p0 ? 1u : 0u) << r;
        bits |= (p1 ? 1u : 0u) << (4 + r);
      }
      if (L < 4) R[t].mask_lo |= bits << (8 * L);
      else R[t].mask_hi = bits;
      if constexpr (N::XYZ) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          f0[t][r] = hh[r] + bc[4 * g + r];
          f1[t][r] = hh[4 + r] + bc[16 + 4 * g + r];
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) R[t].h[j] = hh[j];
      }
    }
    if constexpr (N::XYZ) {
      mm_fwd_t<N::CD / 16, N::LDC, T>(lds + N::WC + L * HID * N::LDC, 0, xc, f0, f1, i, g);
#pragma unroll
      for (int t = 0; t < T; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          R[t].h[r] = f0[t][r];
          R[t].h[4 + r] = f1[t][r];
        }
    }
#pragma unroll
    for (int t = 0; t < T; ++t) {
      if (L == 2) {
#pragma unroll
        for (int j = 0; j < 8; ++j) R[t].h2[j] = R[t].h[j];
      }
      if (rec[t] && keep_h) store_rows<2>(rec[t] + Rec<KIND>::H + HID * L, R[t].h, g);
    }
  }
#pragma unroll
  for (int t = 0; t < T; ++t) {
    if (rec[t]) {
      *reinterpret_cast<uint2*>(rec[t] + Rec<KIND>::M + 2 * g) = uint2{R[t].mask_lo, R[t].mask_hi};
      if (g == 0) *reinterpret_cast<float4*>(rec[t] + Rec<KIND>::PF) = float4{R[t].pf[0], R[t].pf[1], R[t].pf[2], 0.f};
    }
    // output_linear (VALU dot over the point's four lanes)
#pragma unroll
    for (int o = 0; o < 4; ++o) {
      if (o >= (KIND == K_COLOR ? 3 : 1)) { out[t][o] = 0.f; continue; }
      const float* wo = lds + N::WO + o * HID;
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) s = s + wo[feat_of(j, g)] * R[t].h[j];
      out[t][o] = sum_groups(s) + lds[N::BO + o];
    }
  }
}

// ---------------------------------------------------------------------------
// Per-wave forward of one decoder for T 16-point tiles on split-f16 MFMA (NetH image).
// Same record contents and output as wave_forward; every nn.Linear is
// mac_fwd over its 32-column input blocks, each block split once (split8) and
// shared by both 16-row output blocks and, through the weight fragments, by the
// T tiles.
// ---------------------------------------------------------------------------
template <int KIND>
struct WaveIn {
  float c[Net<KIND>::CD / 4];  // grid features (C layout; fine: [fine | middle])
  float pf[3];                 // p.float()
};

template <int KIND, int T>
__device__ __forceinline__ void wave_forward_h(const char* img, int i, int g, const WaveIn<KIND> (&R)[T],
                                               float (&out)[T][4], float* const (&rec)[T], bool keep_h,
                                               float& amax) {
  using N = Net<KIND>;
  using H = NetH<KIND>;
  constexpr int CB = N::CD / 32;
  const float* F = reinterpret_cast<const float*>(img);
  half8 ch[CB][T], cl[CB][T];
#pragma unroll
  for (int b = 0; b < CB; ++b)
#pragma unroll
    for (int t = 0; t < T; ++t) split8(R[t].c + 8 * b, ch[b][t], cl[b][t], amax);
  half8 eh[3][T], el[3][T];  // Fourier features sin(p.float() @ B), XYZ decoders
  if constexpr (N::XYZ) {
    // two features per packed-FP32 instruction (v_pk_mul / v_pk_fma: IEEE per element, so
    // the arguments and the reduction are bit-identical to the scalar form k_mlp_dw
    // recomputes).  The padded B columns 93..95 are 0 in the image: sin(0) = 0 exactly.
    const float* B = F + H::FB;
#pragma unroll
    for (int kb = 0; kb < 3; ++kb)
#pragma unroll
      for (int t = 0; t < T; ++t) {
        float e[8];
        const f2 p0 = f2{R[t].pf[0], R[t].pf[0]}, p1 = f2{R[t].pf[1], R[t].pf[1]}, p2 = f2{R[t].pf[2], R[t].pf[2]};
#pragma unroll
        for (int j = 0; j < 8; j += 2) {
          const int m = 32 * kb + feat_of(j, g);  // m + 1 = feat_of(j + 1, g)
          const f2 b0 = *reinterpret_cast<const f2*>(B + m);
          const f2 b1 = *reinterpret_cast<const f2*>(B + EMBP + m);
          const f2 b2 = *reinterpret_cast<const f2*>(B + 2 * EMBP + m);
          const f2 x = fma2(p2, b2, fma2(p1, b1, p0 * b0));
          const f2 y = fourier_sin2(x);
          e[j] = y.x;
          e[j + 1] = y.y;
        }
        split8(e, eh[kb][t], el[kb][t]);
      }
  }
  unsigned mlo[T], mhi[T];
  float h[T][8];
  half8 xh[T], xl[T];    // split input of the next block (h_L)
  half8 h2h[T], h2l[T];  // split h_2 (skip input of block 3)
#pragma unroll
  for (int t = 0; t < T; ++t) mlo[t] = mhi[t] = 0;
#pragma unroll
  for (int L = 0; L < 5; ++L) {
    // the biases start the accumulators (z = b + W x; the fc_c output adds its own bias)
    const float* bl = F + H::BL + L * HID;
    const float* bc = F + H::BC + L * HID;
    floatx4 hh[T][2], mx[T][2];
#pragma unroll
    for (int t = 0; t < T; ++t) {
      hh[t][0] = bias4(bl, g);
      hh[t][1] = bias4(bl + 16, g);
      mx[t][0] = mx[t][1] = zero4();
    }
    const char* M = img + H::lin_off(L);
    const char* M3 = img + H::lin3_off(L);
    if (L == 0) {
      if constexpr (N::XYZ) {
#pragma unroll
        for (int kb = 0; kb < 3; ++kb) mac_fwd<T>(M, M3, kb, eh[kb], el[kb], hh, mx, i, g);
      } else {
        mac_fwd<T>(M, M3, 0, ch[0], cl[0], hh, mx, i, g);
      }
    } else if (L == 3) {
      if constexpr (N::XYZ) {
#pragma unroll
        for (int kb = 0; kb < 3; ++kb) mac_fwd<T>(M, M3, kb, eh[kb], el[kb], hh, mx, i, g);
        mac_fwd<T>(M, M3, 3, h2h, h2l, hh, mx, i, g);
      } else {
        mac_fwd<T>(M, M3, 0, ch[0], cl[0], hh, mx, i, g);
        mac_fwd<T>(M, M3, 1, h2h, h2l, hh, mx, i, g);
      }
    } else {
      mac_fwd<T>(M, M3, 0, xh, xl, hh, mx, i, g);
    }
    floatx4 fh[T][2], fm[T][2];
    if constexpr (N::XYZ) {
#pragma unroll
      for (int t = 0; t < T; ++t) {
        fh[t][0] = bias4(bc, g);
        fh[t][1] = bias4(bc + 16, g);
        fm[t][0] = fm[t][1] = zero4();
      }
#pragma unroll
      for (int b = 0; b < CB; ++b)
        mac_fwd<T>(img + H::fc_off(L), img + H::fc3_off(L), b, ch[b], cl[b], fh, fm, i, g);
    }
    mfma16_drain();
#pragma unroll
    for (int t = 0; t < T; ++t) {
      unsigned bits = 0;
#pragma unroll
      for (int j = 0; j < 8; j += 2) {
        const int ob = j >> 2, r = j & 3;
        // z = (b + hi.hi) + 2^-11 (hi.lo + (mid + lo3).hi), two features per v_pk_fma
        const f2 z = fma2(f2{mx[t][ob][r], mx[t][ob][r + 1]}, f2{SPLIT_INV, SPLIT_INV},
                          f2{hh[t][ob][r], hh[t][ob][r + 1]});
        const bool p0 = z.x > 0.f, p1 = z.y > 0.f;
        f2 v = f2{p0 ? z.x : 0.f, p1 ? z.y : 0.f};
        bits |= (p0 ? 1u : 0u) << j;
        bits |= (p1 ? 1u : 0u) << (j + 1);
        if constexpr (N::XYZ)
          v = v + fma2(f2{fm[t][ob][r], fm[t][ob][r + 1]}, f2{SPLIT_INV, SPLIT_INV},
                       f2{fh[t][ob][r], fh[t][ob][r + 1]});
        h[t][j] = v.x;
        h[t][j + 1] = v.y;
      }
      if (L < 4) mlo[t] |= bits << (8 * L);
      else mhi[t] = bits;
      if (L < 4) split8(h[t], xh[t], xl[t], amax);
      if (L == 2) {
        h2h[t] = xh[t];
        h2l[t] = xl[t];
      }
      if (rec[t] && keep_h) store_rows<2>(rec[t] + Rec<KIND>::H + HID * L, h[t], g);
    }
  }
#pragma unroll
  for (int t = 0; t < T; ++t) {
    if (rec[t]) {
      *reinterpret_cast<uint2*>(rec[t] + Rec<KIND>::M + 2 * g) = uint2{mlo[t], mhi[t]};
      if (g == 0) *reinterpret_cast<float4*>(rec[t] + Rec<KIND>::PF) = float4{R[t].pf[0], R[t].pf[1], R[t].pf[2], 0.f};
    }
#pragma unroll
    for (int o = 0; o < 4; ++o) {
      if (o >= (KIND == K_COLOR ? 3 : 1)) { out[t][o] = 0.f; continue; }
      const float* wo = F + H::WO + o * HID;
      f2 s2 = f2{0.f, 0.f};
#pragma unroll
      for (int j = 0; j < 8; j += 2) s2 = fma2(*reinterpret_cast<const f2*>(wo + feat_of(j, g)), f2{h[t][j], h[t][j + 1]}, s2);
      out[t][o] = sum_groups(s2.x + s2.y) + F[H::BO + o];
    }
  }
}

// ---------------------------------------------------------------------------
// forward kernel
// ---------------------------------------------------------------------------
// Constant-index select: a dynamic index into the by-value kernel-argument block
// (ctx.jobs[blockIdx.y]) would make the compiler copy the whole block to scratch.
__device__ __forceinline__ Job pick_job(const Job (&jobs)[MAX_JOBS], unsigned y) {
  return y == 0 ? jobs[0] : (y == 1 ? jobs[1] : jobs[2]);
}

// FUSE: the tiles' grid features are gathered here (MLP.sample_grid_feature,
// decoder.py:179-188, and the fine decoder's grid_middle lookup, :196-202: make_corners +
// gather8, the same arithmetic as k_grid_gather) instead of read from cfeat, and the
// backward's gradient buffer is zero-filled at the end of the workgroup's tiles.
// F32: the decoder GEMMs on the exact-f32 MFMA (wave_forward, the f32 LDS image) instead of
// split-f16 (wave_forward_h).  The split-f16 instantiation folds max |operand| of its
// weights and activations into amax and, if any reaches RANGE_LIMIT (nc_device.h), sets
// the job's range flag, so that k_mlp_fwd_exact recomputes the job on the F32 path.
template <int KIND, bool FUSE, bool F32>
__device__ __forceinline__ void fwd_job(const MlpCtx& ctx, const Job& job, int j, float* lds, int64_t wg,
                                        int64_t nwg, bool zero_fill) {
  constexpr int T = FWD_TILES;
  constexpr int CQ = Net<KIND>::CD / 16;
  float amax = 0.f;
  if constexpr (F32)
    load_weights<KIND, PADW_FWD, fwd_threads(FUSE)>(lds, ctx.dec[KIND]);
  else
    copy_wimage<KIND, fwd_threads(FUSE)>(reinterpret_cast<char*>(lds), ctx.wimg + (int64_t)j * WIMG_STRIDE, amax);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
  const int waves = blockDim.x >> 6;
  const int64_t per = 16 * waves * T;  // points per workgroup iteration
  const int64_t nblk = (ctx.P + per - 1) / per;
  // tile t of this wave: points blk*per + (t*waves + wave)*16 + [0, 16)
  auto point = [&](int64_t blk, int t) { return blk * per + (int64_t)(t * waves + wave) * 16 + i; };
  // inputs of the wave's next tiles (p.float() and the grid features) are loaded one
  // iteration ahead, so their latency hides behind the current tiles' MLP
  float4 nf[T];
  float4 nc[T][FUSE ? 1 : CQ];
  float4 nx[T];  // FUSE: normalize_3d_coordinate of the next tiles' points (this decoder's bound)
  auto load_inputs = [&](int64_t blk) {
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const int64_t p = point(blk, t);
      const bool ok = blk < nblk && p < ctx.P;
      nf[t] = ok ? ctx.pf[p] : float4{0.f, 0.f, 0.f, 0.f};
      if constexpr (FUSE) {
        nx[t] = ok ? ctx.xyz[(int64_t)job.slot * ctx.P + p] : float4{0.f, 0.f, 0.f, 0.f};
      } else {
        const float* cf = ctx.cfeat + job.c_off + (ok ? p : 0) * job.c_stride + 4 * g;
#pragma unroll
        for (int q = 0; q < CQ; ++q)
          nc[t][q] = ok ? *reinterpret_cast<const float4*>(cf + 16 * q) : float4{0.f, 0.f, 0.f, 0.f};
      }
    }
  };
  load_inputs(wg);
  for (int64_t blk = wg; blk < nblk; blk += nwg) {
    // keep the (loop-invariant) LDS weight reads inside the loop: hoisting all of
    // them out of the persistent loop would need thousands of registers
    asm volatile("" ::: "memory");
    std::conditional_t<F32, WaveRegs<KIND>, WaveIn<KIND>> R[T];
    float* rec[T];
    int64_t pt[T];
#pragma unroll
    for (int t = 0; t < T; ++t) {
      pt[t] = point(blk, t);
      R[t].pf[0] = nf[t].x; R[t].pf[1] = nf[t].y; R[t].pf[2] = nf[t].z;
      if constexpr (FUSE) {
        const float xyz[3] = {nx[t].x, nx[t].y, nx[t].z};
        // every corner of the tile's lookups in flight at once (the MLP's registers are
        // free here): one memory round trip per tile
        if constexpr (KIND == K_FINE) {  // [fine | middle]: + the no-grad grid_middle lookup
          const nc_grid& G1 = ctx.grids[K_FINE];
          const nc_grid& G2 = ctx.grids[K_MID];
          Corners c1, c2;
          make_corners(G1, xyz, c1);
          make_corners(G2, xyz, c2);
          gather8x2(G1, c1, G2, c2, g, R[t].c, R[t].c + 8);
        } else {
          const nc_grid& G = ctx.grids[KIND];
          Corners co;
          make_corners(G, xyz, co);
          gather8<true>(G, co, g, R[t].c);
        }
      } else {
#pragma unroll
        for (int q = 0; q < CQ; ++q) {
          R[t].c[4 * q + 0] = nc[t][q].x; R[t].c[4 * q + 1] = nc[t][q].y;
          R[t].c[4 * q + 2] = nc[t][q].z; R[t].c[4 * q + 3] = nc[t][q].w;
        }
      }
      rec[t] = (ctx.save_rec && pt[t] < ctx.P) ? ctx.rec + job.rec_off + pt[t] * Rec<KIND>::STRIDE : nullptr;
      if constexpr (FUSE) {  // the features k_mlp_dw reads from the record (k_grid_gather's store)
        if (rec[t]) store_rows<CQ>(rec[t] + Rec<KIND>::C, R[t].c, g);
      }
    }
    load_inputs(blk + nwg);
    float out[T][4];
    if constexpr (F32)
      wave_forward<KIND, T>(lds, i, g, R, out, rec, job.keep_h != 0);
    else
      wave_forward_h<KIND, T>(reinterpret_cast<const char*>(lds), i, g, R, out, rec, job.keep_h != 0, amax);
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const int64_t p = pt[t];
      if (p < ctx.P && g == 0) {
        if constexpr (KIND == K_COLOR) {
          ctx.rgb[p * 3 + 0] = out[t][0];
          ctx.rgb[p * 3 + 1] = out[t][1];
          ctx.rgb[p * 3 + 2] = out[t][2];
        } else {
          ctx.occ[(int64_t)job.slot * ctx.P + p] = out[t][0];
        }
      }
    }
  }
  if constexpr (!F32) {  // out of the f16 range: the whole job is recomputed (rare; one store per lane)
    if (!(amax < RANGE_LIMIT) && ctx.range_flag) ctx.range_flag[j] = 1u;
  }
  if constexpr (FUSE) {  // the backward's gradient buffer (nc_render_args.grad_zero): stores last
    if (zero_fill && ctx.zero_fill) {
      const int64_t nthr = (int64_t)gridDim.x * blockDim.x;
      for (int64_t z = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; z < ctx.zero_n4; z += nthr)
        ctx.zero_fill[z] = float4{0.f, 0.f, 0.f, 0.f};
    }
  }
}

// job of workgroup b in a 1-D grid split [off[0], off[1]), [off[1], off[2]), ...
__device__ __forceinline__ int job_of_wg(const int32_t (&off)[MAX_JOBS + 1], int b) {
  return (b >= off[1] ? 1 : 0) + (b >= off[2] ? 1 : 0);
}

#ifdef NC_MFMA_F32
constexpr bool FWD_F32 = true;   // A/B build: every forward on the exact-f32 MFMA
#else
constexpr bool FWD_F32 = false;
#endif

template <bool FUSE, bool F32, bool EXACT>
__device__ __forceinline__ void fwd_kernel(const MlpCtx& ctx, float* lds) {
  const int b = blockIdx.x;
  const int j = job_of_wg(ctx.fwd_off, b);
  if constexpr (EXACT) {  // k_mlp_fwd_exact: only the jobs whose split-f16 operands left the range
    if (ctx.range_flag == nullptr || ctx.range_flag[j] == 0u) return;
  }
  const Job job = pick_job(ctx.jobs, j);
  const int o0 = j == 0 ? ctx.fwd_off[0] : (j == 1 ? ctx.fwd_off[1] : ctx.fwd_off[2]);
  const int o1 = j == 0 ? ctx.fwd_off[1] : (j == 1 ? ctx.fwd_off[2] : ctx.fwd_off[3]);
  switch (job.kind) {
    case K_COARSE: fwd_job<K_COARSE, FUSE, F32>(ctx, job, j, lds, b - o0, o1 - o0, !EXACT); break;
    case K_MID: fwd_job<K_MID, FUSE, F32>(ctx, job, j, lds, b - o0, o1 - o0, !EXACT); break;
    case K_FINE: fwd_job<K_FINE, FUSE, F32>(ctx, job, j, lds, b - o0, o1 - o0, !EXACT); break;
    default: fwd_job<K_COLOR, FUSE, F32>(ctx, job, j, lds, b - o0, o1 - o0, !EXACT); break;
  }
}

template <bool FUSE>
__global__ void __launch_bounds__(fwd_threads(FUSE)) k_mlp_fwd(const MlpCtx ctx) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  fwd_kernel<FUSE, FWD_F32, false>(ctx, lds);
}

// The range guard's second pass (decoder.py:209-216 in fp32 addmm semantics): right after
// k_mlp_fwd, every workgroup reads its job's range flag and returns at once when it is
// clear (the normal case: one load per workgroup); a flagged job is recomputed whole on
// the exact-f32 MFMA -- outputs, activation records and fused grid features overwritten
// with the f32 path's, which needs no range.  The gradient buffer fill is not repeated.
template <bool FUSE>
__global__ void __launch_bounds__(fwd_threads(FUSE)) k_mlp_fwd_exact(const MlpCtx ctx) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  fwd_kernel<FUSE, true, true>(ctx, lds);
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

// ---------------------------------------------------------------------------
// k_mlp_dx: backward through the decoder per wavefront (16 points), no barriers.
// dh_4 = W_out^T d out; per block L (4..0): dz = dh ⊙ relu'(Z_L); d features +=
// Wc_L^T dh (own 32 channels only); dh_{L-1} / d emb = W_L^T dz (MFMA).  Fourier:
// dx = d emb ⊙ cos(p @ B); d p.float() = B dx.  Writes dh_L and dx for k_mlp_dw,
// d features for k_grid_bwd and the Fourier part of the point gradient.
// ---------------------------------------------------------------------------
__host__ __device__ constexpr int cmax_(int a, int b) { return a > b ? a : b; }
// k_mlp_dx LDS: its weight image, then one grid-scatter slice per wave
constexpr int DX_SLICE_BASE = cmax_(cmax_(Net<K_COARSE, PADW_BWD>::WEIGHTS, Net<K_MID, PADW_BWD>::WEIGHTS),
                                    cmax_(Net<K_FINE, PADW_BWD>::WEIGHTS, Net<K_COLOR, PADW_BWD>::WEIGHTS));
static_assert(DX_SLICE_BASE % 4 == 0, "scatter slices are float4-aligned");
// d B accumulators [wave][3][EMBP]: one private slice per wave (plain adds in a fixed
// order, no LDS atomics), summed over the waves in wave order at the end -- deterministic
constexpr int DX_BACC = DX_SLICE_BASE + (DX_THREADS / 64) * SCAT_FLOATS;
constexpr int DX_LDS_FLOATS = DX_BACC + (DX_THREADS / 64) * DX_BSLAB;
static_assert(DX_LDS_FLOATS * 4 <= 160 * 1024, "dX LDS budget");

// VEC: every grid of the launch is channels-last with float4-aligned rows (the host
// checked), so the strided-channel trilinear path is not compiled in (its per-channel
// offsets were most of the kernel's register spills)
template <int KIND, bool JAC, bool VEC>
__device__ __forceinline__ void dx_job(const MlpCtx& ctx, const Job& job, float* lds) {
  using N = Net<KIND>;
  using RC = Rec<KIND>;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
  const int waves = blockDim.x >> 6;
  const bool need_dw = job.need_dw != 0;
  const bool need_grid = job.need_grid != 0;
  const bool need_coord = job.need_coord != 0;
  const bool need_dc = need_grid || need_coord;
  float* bacc = lds + DX_BACC + wave * DX_BSLAB;  // this wave's d fourier_B (xyz decoders, weight gradients)
  for (int e = threadIdx.x; e < waves * DX_BSLAB; e += blockDim.x) lds[DX_BACC + e] = 0.f;  // ordered by the image copy's barrier
  {  // the f32 image the forward's builders wrote (nc_wimage.h dximg_build), copied flat
    const float4* src = reinterpret_cast<const float4*>(ctx.dximg + (int64_t)blockIdx.y * (DXIMG_STRIDE / 4));
    for (int e = threadIdx.x; e < Net<KIND, PADW_BWD>::WEIGHTS / 4; e += DX_THREADS) reinterpret_cast<float4*>(lds)[e] = src[e];
    __syncthreads();
  }
  // this wave's scatter staging (a scalar base: nothing per lane to keep live across tiles)
  float* slice = lds + DX_SLICE_BASE + __builtin_amdgcn_readfirstlane(wave) * SCAT_FLOATS;
  const int64_t ntiles = (ctx.P + 15) / 16;
  const float dscale = ctx.dout_scale ? (float)*ctx.dout_scale : 1.f;  // fused mapper loss: d loss
  for (int64_t t = (int64_t)blockIdx.x * waves + wave; t < ntiles; t += (int64_t)gridDim.x * waves) {
    asm volatile("" ::: "memory");  // keep LDS weight reads inside the loop (see fwd_job)
    const int64_t p = t * 16 + i;
    const bool valid = p < ctx.P;
    float* rec = ctx.rec + job.rec_off + (valid ? p : 0) * RC::STRIDE;
    float* drec = rec + RC::LEN;
    float dout[4] = {0.f, 0.f, 0.f, 0.f};
    unsigned mlo = 0, mhi = 0;
    if (valid) {
      if constexpr (KIND == K_COLOR) {
        dout[0] = ctx.grgb[p * 3 + 0] * dscale;
        dout[1] = ctx.grgb[p * 3 + 1] * dscale;
        dout[2] = ctx.grgb[p * 3 + 2] * dscale;
      } else {
        dout[0] = ctx.gocc[p] * dscale;
      }
      const uint2 m = *reinterpret_cast<const uint2*>(rec + RC::M + 2 * g);
      mlo = m.x;
      mhi = m.y;
      if (need_dw && g == 0)  // k_mlp_dw reads d out from the record
        *reinterpret_cast<float4*>(drec + RC::DOUT) = float4{dout[0], dout[1], dout[2], 0.f};
    }
    float dh[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float s = 0.f;
#pragma unroll
      for (int o = 0; o < N::NOUT; ++o) s = s + lds[N::WO + o * HID + feat_of(j, g)] * dout[o];
      dh[j] = s;
    }
    floatx4 dc[2] = {zero4(), zero4()};
    floatx4 demb[6] = {zero4(), zero4(), zero4(), zero4(), zero4(), zero4()};
#pragma unroll
    for (int L = 4; L >= 0; --L) {
      if (need_dw && valid) store_rows<2>(drec + RC::DH + HID * L, dh, g);
      float dz[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) dz[j] = mask_bit(mlo, mhi, L, j) ? dh[j] : 0.f;
      if constexpr (N::XYZ) {
        if (need_dc) mm_bwd<2, N::LDC>(lds + N::WC + L * HID * N::LDC, 0, dh, dc, i, g);
      }
      const float* W = lds + N::lin_off(L);
      if (L == 0) {
        if constexpr (N::XYZ) mm_bwd<6, N::LD0>(W, 0, dz, demb, i, g);
        else if (need_dc) mm_bwd<2, N::LD0>(W, 0, dz, dc, i, g);
      } else {
        floatx4 t2[2] = {zero4(), zero4()};
        if (L == 3) {
          if constexpr (N::XYZ) {
            mm_bwd<6, N::LD3>(W, 0, dz, demb, i, g);
            mm_bwd<2, N::LD3>(W, 6, dz, t2, i, g);
          } else {
            if (need_dc) mm_bwd<2, N::LD3>(W, 0, dz, dc, i, g);
            mm_bwd<2, N::LD3>(W, 2, dz, t2, i, g);
          }
        } else {
          mm_bwd<2, N::LDH>(W, 0, dz, t2, i, g);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          dh[r] = t2[0][r];
          dh[4 + r] = t2[1][r];
        }
      }
    }
    float dpf[3] = {0.f, 0.f, 0.f};
    if constexpr (N::XYZ) {
      // dx = d emb * cos(p.float() @ B), produced 4 features at a time and reduced into
      // d p.float() = B dx without keeping all 24 live.  The weight gradient of B,
      // d B[c][m] = sum_points p.float()[c] dx[m] (decoder.py:26-30), is summed here too,
      // instead of 384 B of dx per point written to the record for k_mlp_dw: per 16-feature
      // block t one 16 x 16 product over the tile's 16 points on the MFMA -- four
      // v_mfma_f32_16x16x4_f32 k-steps, A = p.float() of 4 points (rows c, 0 for c >= 3),
      // B = their dx rows transposed through this wave's LDS slice -- whose rows c < 3 are
      // added into the wave's bacc slice (over the workgroup's tiles; summed over the
      // waves in wave order at the end: deterministic).
      const float* B = lds + N::FB;
      const float4 f = valid ? ctx.pf[p] : float4{0.f, 0.f, 0.f, 0.f};
      constexpr int DXB_LD = 24;  // [point][16 features] rows: 16-B aligned, 2 lanes per bank on the reads
      static_assert(16 * DXB_LD <= SCAT_FLOATS, "the d B staging fits the wave's scatter slice");
      float pfa[4];  // A operand of k-step s: p.float()[i] of point 4 s + g (lane i < 3)
      if (need_dw) {
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
          const int src = 4 * s4 + g;  // lane (point 4 s + g, g' = 0)
          const float px = __shfl(f.x, src), py = __shfl(f.y, src), pz = __shfl(f.z, src);
          pfa[s4] = i == 0 ? px : (i == 1 ? py : (i == 2 ? pz : 0.f));
        }
      }
#pragma unroll
      for (int t = 0; t < 6; ++t) {
        float dx4[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = 16 * t + 4 * g + r;
          const float x = __builtin_fmaf(f.z, B[2 * EMBP + m], __builtin_fmaf(f.y, B[EMBP + m], f.x * B[m]));
          dx4[r] = (m < EMB) ? demb[t][r] * fourier_cos(x) : 0.f;
          dpf[0] = dpf[0] + B[m] * dx4[r];
          dpf[1] = dpf[1] + B[EMBP + m] * dx4[r];
          dpf[2] = dpf[2] + B[2 * EMBP + m] * dx4[r];
        }
        if (need_dw) {  // wave-uniform
          *reinterpret_cast<float4*>(slice + i * DXB_LD + 4 * g) = float4{dx4[0], dx4[1], dx4[2], dx4[3]};
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          floatx4 acc = zero4();
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4) acc = mfma4(pfa[s4], slice[(4 * s4 + g) * DXB_LD + i], acc);
          if (g == 0) {  // rows c = 0..2 of the product: feature 16 t + i of d B[c]
#pragma unroll
            for (int c = 0; c < 3; ++c) {
              float* a = bacc + c * EMBP + 16 * t + i;
              *a = *a + acc[c];
            }
          }
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // reads done before block t+1's writes
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
      }
      if (need_coord) {
#pragma unroll
        for (int k = 0; k < 3; ++k) dpf[k] = sum_groups(dpf[k]);
      }
    }
    // trilinear backward of this decoder's own grid lookup (nc_grid.h): coordinate
    // gradient and grid scatter, fused here so the scatter's atomics overlap other
    // waves' MFMA work
    double gg[3] = {0.0, 0.0, 0.0};
    if (need_dc) {
      const nc_grid& G = ctx.grids[KIND];
      const float4 n = valid ? ctx.xyz[(int64_t)job.slot * ctx.P + p] : float4{-1.f, -1.f, -1.f, 0.f};
      const float xyz[3] = {n.x, n.y, n.z};
      Corners co;
      make_corners(G, xyz, co);
      float dcv[8];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        dcv[r] = valid ? dc[0][r] : 0.f;
        dcv[4 + r] = valid ? dc[1][r] : 0.f;
      }
      if (need_coord) {
        float gi[3] = {0.f, 0.f, 0.f};
        if (JAC) {  // the forward's trilinear Jacobian (NC_SAVE_POINT_JACOBIAN): no corner re-reads
          const float* J = ctx.jac + ((int64_t)job.slot * ctx.P + (valid ? p : 0)) * 96 + 4 * g;
#pragma unroll
          for (int a = 0; a < 3; ++a) {
            const float4 lo = *reinterpret_cast<const float4*>(J + 32 * a);
            const float4 hi = *reinterpret_cast<const float4*>(J + 32 * a + 16);
            gi[a] = lo.x * dcv[0] + lo.y * dcv[1] + lo.z * dcv[2] + lo.w * dcv[3] +
                    hi.x * dcv[4] + hi.y * dcv[5] + hi.z * dcv[6] + hi.w * dcv[7];
          }
        } else if (VEC || grid_vec_ok(G)) {
          grid_coord_grad<true>(G, co, dcv, g, gi);
        } else {
          if constexpr (!VEC) grid_coord_grad<false>(G, co, dcv, g, gi);
        }
        const float gm[3] = {co.gmx, co.gmy, co.gmz};
        const nc_decoder_params& D = ctx.dec[KIND];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          // normalize_3d_coordinate backward: (g * 2) / (hi - lo)
          const float gk = sum_groups(gi[k]) * gm[k];
          gg[k] = ((double)gk * 2.0) / (D.bound[k][1] - D.bound[k][0]);
        }
        // the point gradient leaves before the scatter (its registers are free across the
        // scatter walk's loop)
        if (valid && g == 0) {
          double* dst = ctx.dpts + ((int64_t)job.slot * ctx.P + p) * 3;
#pragma unroll
          for (int k = 0; k < 3; ++k) dst[k] = gg[k] + (double)dpf[k];
        }
      }
      if (need_grid) {
        if (ctx.dfeat) {  // NC_DETERMINISTIC: ordered reduction in nc_det.hip instead of atomics
          if (valid) {
            float* df = ctx.dfeat + ((int64_t)job.slot * ctx.P + p) * 32;
            *reinterpret_cast<float4*>(df + 4 * g) = float4{dcv[0], dcv[1], dcv[2], dcv[3]};
            *reinterpret_cast<float4*>(df + 16 + 4 * g) = float4{dcv[4], dcv[5], dcv[6], dcv[7]};
          }
        } else {
          grid_scatter(G, co, dcv, valid, slice, i, g, lane);
        }
      }
    }
  }
  if constexpr (N::XYZ) {  // this workgroup's d B partial -> its bslab row (k_mlp_dw folds the rows into its slab)
    if (need_dw && ctx.bslab) {
      __syncthreads();
      float* row = ctx.bslab + ((int64_t)blockIdx.y * ctx.bslab_rows + blockIdx.x) * DX_BSLAB;
      for (int e = threadIdx.x; e < DX_BSLAB; e += blockDim.x) {
        float sum = 0.f;
        for (int w = 0; w < waves; ++w) sum = sum + lds[DX_BACC + w * DX_BSLAB + e];
        row[e] = sum;
      }
    }
  }
}

// JAC: the coordinate gradient from the forward's saved Jacobian (NC_SAVE_POINT_JACOBIAN);
// its own instantiation, so the corner re-read path's registers do not weigh on it
template <bool JAC, bool VEC>
__global__ void __launch_bounds__(DX_THREADS) k_mlp_dx(const MlpCtx ctx) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const Job job = pick_job(ctx.jobs, blockIdx.y);
  if (!job.need_dw && !job.need_grid && !job.need_coord) return;
  switch (job.kind) {
    case K_COARSE: dx_job<K_COARSE, JAC, VEC>(ctx, job, lds); break;
    case K_MID: dx_job<K_MID, JAC, VEC>(ctx, job, lds); break;
    case K_FINE: dx_job<K_FINE, JAC, VEC>(ctx, job, lds); break;
    default: dx_job<K_COLOR, JAC, VEC>(ctx, job, lds); break;
  }
}

// ---------------------------------------------------------------------------
// k_mlp_dw: weight gradients dW = sum_points dY^T X as a streamed GEMM.
// Each workgroup walks 32-point sub-chunks of one decoder: the points' forward
// and backward records are copied contiguously into LDS ([point][record] rows,
// row length == 16 mod 32 floats -> conflict-free ds_read_b32 operands), then
// every dW tile of every layer (16x16, table DwTiles) is advanced by 8 MFMA
// k-steps of 4 points.  Tiles are owned by waves for the whole kernel and kept in
// registers; bias gradients (row sums of dY) go to LDS float atomics.  One flush
// per workgroup into a slab, summed by k_param_reduce.
// ---------------------------------------------------------------------------
#ifndef NC_DW_NPTS
#define NC_DW_NPTS 16
#endif
constexpr int DW_NPTS = NC_DW_NPTS;  // points per staged sub-chunk (4 MFMA k-steps; 16 vs 32: dw -2.5 us at C2 with the 656-B backward record, profiles/r03/ab_dw_shapes.log)

template <int KIND>
struct DwLayout {
  using RC = Rec<KIND>;
  // row: [emb 96 (xyz decoders, recomputed)] [forward record] [backward record] [dZ]
  static constexpr int EMB = 0;
  static constexpr int REC0 = Net<KIND>::XYZ ? EMBP : 0;
  static constexpr int H = REC0 + RC::H;
  static constexpr int C = REC0 + RC::C;
  static constexpr int M = REC0 + RC::M;
  static constexpr int DREC = REC0 + RC::LEN;    // backward record follows the forward one
  static constexpr int PF = REC0 + RC::PF;       // p.float() (4)
  static constexpr int DOUT = DREC + RC::DOUT;   // d out (4; rows >= NOUT zero)
  static constexpr int DZ = DREC + RC::DLEN;     // dZ_L = dh_L * relu'(Z_L), 5 x 32 (staged)
  static constexpr int RS = DZ + 5 * HID;        // row stride (== 16 mod 32)
  static constexpr int BUF = DW_NPTS * RS;
  static constexpr int BACC = BUF;               // bias accumulators after the buffer
  static constexpr int BACC_FLOATS = 16 + 32 * 10;
  static constexpr int FB = BACC + BACC_FLOATS;  // Fourier B [3][96] (xyz decoders)
  static constexpr int TOTAL = FB + 3 * EMBP;
  static_assert(RS % 32 == 16, "row stride must be 16 mod 32 for conflict-free operand reads");
};

// dW tile list of a decoder: phase ids as PhaseMap (0 out, 1..5 lin L=5-ph, 6..10 fc
// L=10-ph, 11 Fourier B); (to, ti) = 16-row block of dY, 16-column block of X.
template <int KIND>
struct DwTiles {
  using N = Net<KIND>;
  static constexpr int NC0 = N::IN0 / 16, NC3 = N::IN3 / 16, NCC = N::CD / 16;
  __host__ __device__ static constexpr int ncols(int ph) {
    return ph == 0 ? 2 : ph == 1 ? 2 : ph == 2 ? NC3 : ph == 3 ? 2 : ph == 4 ? 2 : ph == 5 ? NC0 : ph <= 10 ? NCC : 1;
  }
  __host__ __device__ static constexpr int nrows(int ph) { return ph == 0 ? 1 : ph <= 10 ? 2 : 6; }
  // phase 11 (Fourier B) is summed by k_mlp_dx (DX_BSLAB rows), not here
  __host__ __device__ static constexpr bool present(int ph) { return ph <= 5 || (N::XYZ && ph <= 10); }
  __host__ __device__ static constexpr int count() {
    int n = 0;
    for (int ph = 0; ph < 12; ++ph)
      if (present(ph)) n += nrows(ph) * ncols(ph);
    return n;
  }
  static constexpr int NT = count();
  // packed (ph | to << 8 | ti << 16) of tile tau (branch-free selects, no stack)
  __device__ __forceinline__ static int code(int tau) {
    int res = 0, base = 0;
#pragma unroll
    for (int q = 0; q < 12; ++q) {
      if (!present(q)) continue;
      const int n = nrows(q) * ncols(q);
      const int t = tau - base;
      res = (t >= 0 && t < n) ? (q | ((t / ncols(q)) << 8) | ((t % ncols(q)) << 16)) : res;
      base += n;
    }
    return res;
  }
  __device__ __forceinline__ static void get(int tau, int& ph, int& to, int& ti) {
    const int c = code(tau);
    ph = c & 255;
    to = (c >> 8) & 255;
    ti = c >> 16;
  }
};

constexpr int DW_WAVES = DW_THREADS / 64;

template <int KIND>
__device__ __forceinline__ void dw_job(const MlpCtx& ctx, const Job& job, int j, float* lds, int64_t wg, int64_t nwg) {
  using N = Net<KIND>;
  using RC = Rec<KIND>;
  using LY = DwLayout<KIND>;
  using TL = DwTiles<KIND>;
  constexpr int NS = (TL::NT + DW_WAVES - 1) / DW_WAVES;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
  float* buf = lds;
  float* bacc = lds + LY::BACC;
  for (int e = threadIdx.x; e < LY::BACC_FLOATS; e += blockDim.x) bacc[e] = 0.f;
  if constexpr (N::XYZ) {
    const float* Bsrc = KIND == K_MID ? ctx.dec[K_MID].fourier_B
                        : KIND == K_FINE ? ctx.dec[K_FINE].fourier_B : ctx.dec[K_COLOR].fourier_B;
    for (int e = threadIdx.x; e < 3 * EMBP; e += blockDim.x) {
      const int k = e / EMBP, m = e - k * EMBP;
      lds[LY::FB + e] = m < EMB ? Bsrc[k * EMB + m] : 0.f;
    }
  }
  floatx4 acc[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) acc[s] = zero4();
  // Per-tile operand descriptors.  The k-step is branch-free: a dY column that does
  // not exist (output rows >= NOUT), the Fourier tile's x columns >= 3 and padding
  // slots read the always-zero DOUT+3 slot; relu masks are pre-applied (DZ).
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  // operand row pointers (lane-group g's point row; k-step q adds 4 rows) and mask bit
  int yrow[NS], xrow[NS];  // float offsets into buf (32-bit LDS addresses)
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int tau = wv + DW_WAVES * s;
    int ph, to, ti;
    TL::get(tau < TL::NT ? tau : 0, ph, to, ti);
    const int o = 16 * to + i;
    int yoff, xoff;
    if (ph == 0) {
      yoff = LY::DOUT + (o < N::NOUT ? o : 3);
      xoff = LY::H + HID * 4 + 16 * ti + i;
    } else if (ph <= 5) {
      const int L = 5 - ph;
      yoff = LY::DZ + HID * L + o;
      const int c = 16 * ti + i;
      if (L == 0) xoff = N::XYZ ? LY::EMB + c : LY::C + c;
      else if (L == 3) xoff = N::XYZ ? (c < EMBP ? LY::EMB + c : LY::H + HID * 2 + (c - EMBP))
                                     : (c < HID ? LY::C + c : LY::H + HID * 2 + (c - HID));
      else xoff = LY::H + HID * (L - 1) + c;
    } else if (ph <= 10) {
      yoff = LY::DREC + RC::DH + HID * (10 - ph) + o;
      xoff = LY::C + 16 * ti + i;
    } else {  // not a dW tile here (DwTiles::present)
      yoff = xoff = LY::DOUT + 3;
    }
    if (tau >= TL::NT) yoff = xoff = LY::DOUT + 3;  // padding slot: zero operands, never flushed
    yrow[s] = g * LY::RS + yoff;
    xrow[s] = g * LY::RS + xoff;
  }
  // bias gradients (column sums of dY over the points): thread e < BACC_FLOATS owns bias e
  // (bacc order) and adds its column of every staged sub-chunk in point order, in float64.
  // A bias gradient cancels heavily over the points (sum_p d out_p of an occupancy decoder):
  // the former float32 per-lane sums inside the k-steps were 70x less accurate than the
  // reference's pairwise sum (tests/test_gpu_elementwise.py), and kept NS more VGPRs live
  int bcol = -1;  // the owned bias's column in a staged row
  if (threadIdx.x < LY::BACC_FLOATS) {
    const int e = threadIdx.x;
    const int ph = e < 16 ? 0 : 1 + (e - 16) / 32, row = e < 16 ? e : (e - 16) % 32;
    if (ph == 0) bcol = row < N::NOUT ? LY::DOUT + row : -1;
    else if (ph <= 5) bcol = LY::DZ + HID * (5 - ph) + row;
    else if (N::XYZ) bcol = LY::DREC + RC::DH + HID * (10 - ph) + row;
  }
  double bsum = 0.0;
  // ---- staging: the records of the next sub-chunk are prefetched into registers
  // (branch-free, PER float4 per thread) while the current one is consumed ----
  // A sub-chunk's records are one contiguous block of DW_NPTS * STRIDE floats: item k
  // of this thread is float4 (threadIdx.x + k * DW_THREADS) of the block.
  constexpr int W4 = RC::STRIDE / 4;
  constexpr int ITEMS = DW_NPTS * W4;
  constexpr int PER = (ITEMS + DW_THREADS - 1) / DW_THREADS;
  const int64_t nsub = (ctx.P + DW_NPTS - 1) / DW_NPTS;
  const float4* recs = reinterpret_cast<const float4*>(ctx.rec + job.rec_off);
  int dst[PER];  // LDS destination of item k (fixed for the whole kernel)
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int e = threadIdx.x + k * DW_THREADS;
    const int r = e / W4, c = e - r * W4;
    dst[k] = e < ITEMS ? r * LY::RS + LY::REC0 + 4 * c : -1;
  }
  // the next sub-chunk's records are prefetched into registers while the current
  // one is consumed
  float4 pre[PER];
  auto prefetch = [&](int64_t sub) {
    const float4* blk = recs + sub * DW_NPTS * W4;
    const int64_t lim = (ctx.P - sub * DW_NPTS) * W4;  // valid float4s in this block
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int e = threadIdx.x + k * DW_THREADS;
      pre[k] = (e < ITEMS && e < lim) ? blk[e] : float4{0.f, 0.f, 0.f, 0.f};
    }
  };
  if (wg < nsub) prefetch(wg);
  for (int64_t sub = wg; sub < nsub; sub += nwg) {
    __syncthreads();  // previous sub-chunk's reads are done
    const int64_t p0 = sub * DW_NPTS;
#pragma unroll
    for (int k = 0; k < PER; ++k)
      if (dst[k] >= 0) *reinterpret_cast<float4*>(buf + dst[k]) = pre[k];
    __syncthreads();
    if constexpr (N::XYZ) {  // Fourier features, exactly as wave_forward computes them
      // (rows past P hold p = 0 and padded B columns are 0: sin(0) = 0, no checks)
      const float* B = lds + LY::FB;
      for (int e = threadIdx.x; e < DW_NPTS * EMBP; e += DW_THREADS) {
        const int r = e / EMBP, m = e - r * EMBP;
        const float4 f = *reinterpret_cast<const float4*>(buf + r * LY::RS + LY::PF);
        buf[r * LY::RS + LY::EMB + m] =
            fourier_sin(__builtin_fmaf(f.z, B[2 * EMBP + m], __builtin_fmaf(f.y, B[EMBP + m], f.x * B[m])));
      }
    }
    // dZ_L = dh_L * relu'(Z_L) (mask bit 8L+j of lane-group g's word; L = 4: hi word)
    for (int e = threadIdx.x; e < DW_NPTS * 40; e += DW_THREADS) {
      const int r = e / 40, c4 = e - r * 40, L = c4 >> 3, jj = c4 & 7;
      float* row = buf + r * LY::RS;
      const float4 dh = *reinterpret_cast<const float4*>(row + LY::DREC + RC::DH + HID * L + 4 * jj);
      const unsigned w = __float_as_uint(row[LY::M + 2 * (jj & 3) + (L == 4 ? 1 : 0)]) >>
                         ((L == 4 ? 0 : 8 * L) + 4 * (jj >> 2));
      *reinterpret_cast<float4*>(row + LY::DZ + HID * L + 4 * jj) =
          float4{(w & 1u) ? dh.x : 0.f, (w & 2u) ? dh.y : 0.f, (w & 4u) ? dh.z : 0.f, (w & 8u) ? dh.w : 0.f};
    }
    __syncthreads();
    if (sub + nwg < nsub) prefetch(sub + nwg);
    if (bcol >= 0) {  // rows past P are zero-filled: they add 0
#pragma unroll
      for (int r = 0; r < DW_NPTS; ++r) bsum += (double)buf[r * LY::RS + bcol];
    }
    // ---- tiles: DW_NPTS/4 k-steps of 4 points; the wave's NS accumulation chains are
    // interleaved (k-step outer) so no MFMA waits on its predecessor's result ----
    // one k-step = NS independent MFMAs + 2 NS reads at immediate offsets; unrolled by
    // 4 with a scheduling barrier per k-step (fully unrolled, the scheduler hoists
    // every k-step's reads and spills)
    // A wave whose last tile slot is padding (tau >= NT: 12 of 80 slots for the middle /
    // colour decoders, 8 of 96 for fine) runs NS - 1 chains: the branch is wave-uniform
    // and each SIMD then carries fewer MFMAs per sub-chunk.
    auto ksteps = [&](auto nchains) {
      constexpr int NC = decltype(nchains)::value;
#pragma unroll 4
      for (int q = 0; q < DW_NPTS / 4; ++q) {
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int s = 0; s < NC; ++s) {
          const float av = buf[yrow[s] + 4 * q * LY::RS];
          acc[s] = mfma4(av, buf[xrow[s] + 4 * q * LY::RS], acc[s]);
        }
      }
    };
    if constexpr (NS > 1) {
      if (wv + DW_WAVES * (NS - 1) < TL::NT) ksteps(std::integral_constant<int, NS>{});
      else ksteps(std::integral_constant<int, NS - 1>{});
    } else {
      ksteps(std::integral_constant<int, NS>{});
    }
  }
  if (bcol >= 0) bacc[threadIdx.x] = (float)bsum;
  // ---- flush: every weight-gradient element is owned by exactly one lane and
  // every bias by one bacc entry, so the slab row is written without an image ----
  float* slab = ctx.slab + (int64_t)blockIdx.x * ctx.slab_stride;  // one row per workgroup
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int tau = wv + DW_WAVES * s;
    if (tau >= TL::NT) continue;
    int ph, to, ti;
    TL::get(tau, ph, to, ti);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t idx = PhaseMap<KIND>::w_index(ph, 16 * to + 4 * g + r, 16 * ti + i);
      if (idx >= 0) slab[idx] = acc[s][r];
    }
  }
  __syncthreads();
  for (int e = threadIdx.x; e < LY::BACC_FLOATS; e += blockDim.x) {
    const int ph = e < 16 ? 0 : 1 + (e - 16) / 32;
    const int row = e < 16 ? e : (e - 16) % 32;
    if (ph > 5 && !N::XYZ) continue;
    const int64_t bi = PhaseMap<KIND>::b_index(ph, row);
    if (bi >= 0) slab[bi] = bacc[e];
  }
  if constexpr (N::XYZ) {  // fourier_B: k_mlp_dx's per-workgroup rows wg, wg + nwg, ... summed in order
    if (ctx.bslab) {
      const float* bs = ctx.bslab + (int64_t)j * ctx.bslab_rows * DX_BSLAB;
      for (int e = threadIdx.x; e < 3 * EMB; e += blockDim.x) {
        const int c = e / EMB, m = e - c * EMB;
        float sum = 0.f;
        for (int64_t r = wg; r < ctx.bslab_rows; r += nwg) sum = sum + bs[r * DX_BSLAB + c * EMBP + m];
        slab[N::P_B + e] = sum;
      }
    }
  }
}


__global__ void __launch_bounds__(DW_THREADS) k_mlp_dw(const MlpCtx ctx) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int b = blockIdx.x;
  const int j = job_of_wg(ctx.dw_off, b);
  const Job job = pick_job(ctx.jobs, j);
  if (!job.need_dw) return;
  const int o0 = j == 0 ? ctx.dw_off[0] : (j == 1 ? ctx.dw_off[1] : ctx.dw_off[2]);
  const int o1 = j == 0 ? ctx.dw_off[1] : (j == 1 ? ctx.dw_off[2] : ctx.dw_off[3]);
  switch (job.kind) {
    case K_COARSE: dw_job<K_COARSE>(ctx, job, j, lds, b - o0, o1 - o0); break;
    case K_MID: dw_job<K_MID>(ctx, job, j, lds, b - o0, o1 - o0); break;
    case K_FINE: dw_job<K_FINE>(ctx, job, j, lds, b - o0, o1 - o0); break;
    default: dw_job<K_COLOR>(ctx, job, j, lds, b - o0, o1 - o0); break;
  }
}

// ---------------------------------------------------------------------------
// launch wrappers / layout queries
// ---------------------------------------------------------------------------
__host__ __device__ constexpr int cmax(int a, int b) { return a > b ? a : b; }
constexpr int FWD_F32_LDS_FLOATS =
    cmax(cmax(Net<K_COARSE, PADW_FWD>::WEIGHTS, Net<K_MID, PADW_FWD>::WEIGHTS),
         cmax(Net<K_FINE, PADW_FWD>::WEIGHTS, Net<K_COLOR, PADW_FWD>::WEIGHTS));
constexpr int FWD_LDS_FLOATS =
    FWD_F32 ? FWD_F32_LDS_FLOATS
            : cmax(cmax(NetH<K_COARSE>::BYTES, NetH<K_MID>::BYTES), cmax(NetH<K_FINE>::BYTES, NetH<K_COLOR>::BYTES)) / 4;
static_assert(FWD_F32_LDS_FLOATS * 4 <= 160 * 1024, "f32 weight image LDS budget");
constexpr int DW_LDS_FLOATS = cmax(cmax(DwLayout<K_COARSE>::TOTAL, DwLayout<K_MID>::TOTAL),
                                   cmax(DwLayout<K_FINE>::TOTAL, DwLayout<K_COLOR>::TOTAL));
static_assert(FWD_LDS_FLOATS * 4 <= 160 * 1024, "weight image LDS budget");
static_assert(DW_LDS_FLOATS * 4 <= 160 * 1024, "dW staging LDS budget");

int mlp_fwd_lds_bytes() { return FWD_LDS_FLOATS * 4; }
int mlp_fwd_exact_lds_bytes() { return FWD_F32_LDS_FLOATS * 4; }
int mlp_dw_lds_bytes() { return DW_LDS_FLOATS * 4; }
int64_t max_param_count() {
  return cmax(cmax((int)Net<K_COARSE>::NPARAM, (int)Net<K_MID>::NPARAM),
              cmax((int)Net<K_FINE>::NPARAM, (int)Net<K_COLOR>::NPARAM));
}
int rec_feat_offset(int kind) {
  switch (kind) {
    case K_COARSE: return Rec<K_COARSE>::C;
    case K_MID: return Rec<K_MID>::C;
    case K_FINE: return Rec<K_FINE>::C;
    default: return Rec<K_COLOR>::C;
  }
}

int rec_stride(int kind) {
  switch (kind) {
    case K_COARSE: return Rec<K_COARSE>::STRIDE;
    case K_MID: return Rec<K_MID>::STRIDE;
    case K_FINE: return Rec<K_FINE>::STRIDE;
    default: return Rec<K_COLOR>::STRIDE;
  }
}


template <typename K>
static int set_lds(K kernel, int bytes) {
  return (int)hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}

// resident workgroups per CU of k_mlp_fwd (0; fused gather: 3), k_mlp_dx (1), k_mlp_dw (2), from the
// HIP occupancy calculator (registers, LDS, wave slots); cached per device
int mlp_blocks_per_cu(int which) {
  static int cache[64][4] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64 || which < 0 || which > 3) return 1;
  if (!cache[dev][which]) {
    int n = 0;
    hipError_t e = hipSuccess;
    if (which == 0) {
      set_lds(k_mlp_fwd<false>, mlp_fwd_lds_bytes());
      e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_mlp_fwd<false>, FWD_THREADS, mlp_fwd_lds_bytes());
    } else if (which == 3) {
      set_lds(k_mlp_fwd<true>, mlp_fwd_lds_bytes());
      e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_mlp_fwd<true>, FWD_THREADS_FUSED, mlp_fwd_lds_bytes());
    } else if (which == 1) {
      set_lds(k_mlp_dx<true, false>, mlp_dx_lds_bytes());
      set_lds(k_mlp_dx<false, false>, mlp_dx_lds_bytes());
      set_lds(k_mlp_dx<false, true>, mlp_dx_lds_bytes());
      e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_mlp_dx<true, false>, DX_THREADS, mlp_dx_lds_bytes());
    } else {
      set_lds(k_mlp_dw, mlp_dw_lds_bytes());
      e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_mlp_dw, DW_THREADS, mlp_dw_lds_bytes());
    }
    cache[dev][which] = (e == hipSuccess && n > 0) ? n : 1;
  }
  return cache[dev][which];
}

int decoder_macs(int kind) {  // SURVEY.md §8a a10-a11 (MAC per point)
  switch (kind) {
    case K_COARSE: return 6176;
    case K_MID: return 15479;
    case K_FINE: return 20599;
    default: return 15575;
  }
}

// k_mlp_fwd on split-f16 MFMA is no longer MAC-bound: per tile the Fourier
// features, the operand splits and the record stores cost about the same for the
// three xyz decoders, the fine decoder's second feature block a little more
int fwd_tile_cost(int kind) {
#if defined(NC_MFMA_F32)
  return decoder_macs(kind);
#else
  switch (kind) {
    case K_COARSE: return 40;
    case K_FINE: return 112;
    default: return 100;
  }
#endif
}

#ifndef NC_EXACT_WGS
#define NC_EXACT_WGS 16
#endif
constexpr int EXACT_WGS_PER_JOB = NC_EXACT_WGS;

int launch_mlp_fwd(const MlpCtx& c, hipStream_t s) {
  static int attr = -1;
  if (attr != 0 && (attr = set_lds(k_mlp_fwd<false>, mlp_fwd_lds_bytes()) |
                           set_lds(k_mlp_fwd<true>, mlp_fwd_lds_bytes())) != 0)
    return attr;
  static int attr_x = -1;
  if (attr_x != 0 && (attr_x = set_lds(k_mlp_fwd_exact<false>, mlp_fwd_exact_lds_bytes()) |
                               set_lds(k_mlp_fwd_exact<true>, mlp_fwd_exact_lds_bytes())) != 0)
    return attr_x;
  const dim3 grid(c.fwd_off[c.n_jobs]);
  if (c.fuse_gather)
    hipLaunchKernelGGL(k_mlp_fwd<true>, grid, dim3(FWD_THREADS_FUSED), mlp_fwd_lds_bytes(), s, c);
  else
    hipLaunchKernelGGL(k_mlp_fwd<false>, grid, dim3(FWD_THREADS), mlp_fwd_lds_bytes(), s, c);
  if (hipError_t e = hipGetLastError()) return (int)e;
  if (FWD_F32 || c.range_flag == nullptr) return 0;
  // the recompute pass runs on a few workgroups per job: its normal cost is the dispatch
  // of workgroups that read one flag and return (4.7 us for the forward's 256 x 512
  // threads at C2, rocprofv3), and a flagged job -- never seen with sane inputs -- takes a
  // few times the forward's time instead of one
  MlpCtx x = c;
  for (int j = 0; j <= MAX_JOBS; ++j) x.fwd_off[j] = (j < c.n_jobs ? j : c.n_jobs) * EXACT_WGS_PER_JOB;
  const dim3 xgrid(x.fwd_off[c.n_jobs]);
  if (c.fuse_gather)
    hipLaunchKernelGGL(k_mlp_fwd_exact<true>, xgrid, dim3(FWD_THREADS_FUSED), mlp_fwd_exact_lds_bytes(), s, x);
  else
    hipLaunchKernelGGL(k_mlp_fwd_exact<false>, xgrid, dim3(FWD_THREADS), mlp_fwd_exact_lds_bytes(), s, x);
  return (int)hipGetLastError();
}

int mlp_dx_lds_bytes() { return DX_LDS_FLOATS * 4; }

int launch_mlp_dx(const MlpCtx& c, int grid_x, bool vec, hipStream_t s) {
  static int attr = -1;
  if (attr != 0 && (attr = set_lds(k_mlp_dx<true, false>, mlp_dx_lds_bytes()) |
                           set_lds(k_mlp_dx<false, false>, mlp_dx_lds_bytes()) |
                           set_lds(k_mlp_dx<false, true>, mlp_dx_lds_bytes())) != 0)
    return attr;
  const dim3 grid(grid_x, c.n_jobs);
  if (c.jac)
    hipLaunchKernelGGL((k_mlp_dx<true, false>), grid, dim3(DX_THREADS), mlp_dx_lds_bytes(), s, c);
  else if (vec)
    hipLaunchKernelGGL((k_mlp_dx<false, true>), grid, dim3(DX_THREADS), mlp_dx_lds_bytes(), s, c);
  else
    hipLaunchKernelGGL((k_mlp_dx<false, false>), grid, dim3(DX_THREADS), mlp_dx_lds_bytes(), s, c);
  return (int)hipGetLastError();
}

int launch_mlp_dw(const MlpCtx& c, hipStream_t s) {
  static int attr = -1;
  if (attr != 0 && (attr = set_lds(k_mlp_dw, mlp_dw_lds_bytes())) != 0) return attr;
  hipLaunchKernelGGL(k_mlp_dw, dim3(c.dw_off[c.n_jobs]), dim3(DW_THREADS), mlp_dw_lds_bytes(), s, c);
  return (int)hipGetLastError();
}

}  // namespace nc
