// nc_imap.hip — the iMAP* scene MLP (configs/imap.yaml).
//
// get_model(nice=False) (src/conv_onet/config.py:28-32) builds one MLP with
// c_dim = 0, hidden 256, 4 blocks, no skip, colour output (decoder.py:116-219):
//   emb = sin(p.float() @ B)                       [P, 93]   (decoder.py:26-30)
//   h_0 = relu(emb W_0^T + b_0), h_l = relu(h_{l-1} W_l^T + b_l)   [P, 256]
//   raw = h_3 W_out^T + b_out                      [P, 4]
// Unlike the 32-wide NICE decoders (whole network in one wavefront's registers,
// nc_mlp.hip), every layer here is a 256-wide GEMM with 65k MACs per point, so
// each layer is one launch of an LDS-tiled f32 MFMA GEMM (v_mfma_f32_16x16x4_f32,
// exact f32 products like the reference's fp32 addmm) with the bias / ReLU /
// ReLU-mask epilogue fused:
//   forward   h_l   = relu(h_{l-1} W_l^T + b_l)          (A point-major, B = W [n][k])
//   backward  dz_l  = (dz_{l+1} W_{l+1}) . [h_l > 0]      (B = W [k][n])
//   weights   dW_l  = dz_l^T h_{l-1}                      (split over points, float atomics)
// plus the Fourier embedding (forward / backward) and the bias column sums.
// Activations stay point-major [P][256] in HBM (1 KB per point per layer); at
// 512 FLOP per 4-byte activation read per layer the GEMMs are MFMA-bound.
#include <hip/hip_runtime.h>

#include "nc_device.h"
#include "nc_internal.h"

namespace nc {

#ifndef NC_IMAP_GT_K
#define NC_IMAP_GT_K 16
#endif
#ifndef NC_IMAP_WT
#define NC_IMAP_WT 2
#endif
// workgroup tile: 2 x 2 waves, each WT x WT blocks of 16 x 16; k-slice GT_K
constexpr int WT = NC_IMAP_WT;
constexpr int GT_M = 32 * WT, GT_N = 32 * WT, GT_K = NC_IMAP_GT_K;
static_assert(GT_K % 16 == 0 && GT_K <= 64, "k-slice: whole 16-float rows per thread group");
static_assert(GT_M * GT_K % 256 == 0 && GT_M <= 256, "operand tile loads: whole elements per thread");
constexpr int GT_LD = GT_M + 4;                 // LDS row pad

// C[m][n] (+)= sum_k A(m,k) B(k,n)
//   A_KM: A(m,k) = A[k*lda + m]   else A[m*lda + k]
//   B_KN: B(k,n) = B[k*ldb + n]   else B[n*ldb + k]
// epilogue: + bias[n]; relu; * (mask[m*ldm + n] > 0); atomic accumulate (split-K).
// one k-slice of the wave's (16 WT) x (16 WT) sub-tile: WT x WT blocks of v_mfma_f32_16x16x4_f32
__device__ __forceinline__ void slice_mfma(const float (&As)[GT_K][GT_LD], const float (&Bs)[GT_K][GT_LD], int wm,
                                           int wn, int i, int q, floatx4 (&acc)[WT][WT]) {
#pragma unroll
  for (int kk = 0; kk < GT_K; kk += 4) {
    float a[WT], b[WT];
#pragma unroll
    for (int u = 0; u < WT; ++u) {
      a[u] = As[kk + q][wm + 16 * u + i];
      b[u] = Bs[kk + q][wn + 16 * u + i];
    }
#pragma unroll
    for (int bm = 0; bm < WT; ++bm)
#pragma unroll
      for (int bn = 0; bn < WT; ++bn) acc[bm][bn] = mfma4(a[bm], b[bn], acc[bm][bn]);
  }
}

template <bool A_KM, bool B_KN>
__global__ void __launch_bounds__(256) k_imap_gemm(const ImapGemm g) {
  __shared__ float As[GT_K][GT_LD];
  __shared__ float Bs[GT_K][GT_LD];
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63, i = lane & 15, q = lane >> 4;
  const int64_t m0 = (int64_t)blockIdx.x * GT_M;
  const int64_t n0 = (int64_t)blockIdx.y * GT_N;
  const int64_t kb = (int64_t)blockIdx.z * g.k_split;
  const int64_t ke = kb + g.k_split < g.K ? kb + g.k_split : g.K;
  const int wm = (wave & 1) * 16 * WT, wn = (wave >> 1) * 16 * WT;
  floatx4 acc[WT][WT];
#pragma unroll
  for (int bm = 0; bm < WT; ++bm)
#pragma unroll
    for (int bn = 0; bn < WT; ++bn) acc[bm][bn] = zero4();
  for (int64_t k0 = kb; k0 < ke; k0 += GT_K) {
#pragma unroll
    for (int j = 0; j < GT_M * GT_K / 256; ++j) {  // GT_M x GT_K elements of each operand tile
      int kk, mm;
      if (A_KM) { mm = t % GT_M; kk = t / GT_M + (256 / GT_M) * j; } else { kk = t % GT_K; mm = t / GT_K + (256 / GT_K) * j; }
      const int64_t gk = k0 + kk, gm = m0 + mm;
      float v = 0.f;
      if (gk < ke && gm < g.M) v = A_KM ? g.A[gk * g.lda + gm] : g.A[gm * g.lda + gk];
      As[kk][mm] = v;
      int kn, nn;
      if (B_KN) { nn = t % GT_N; kn = t / GT_N + (256 / GT_N) * j; } else { kn = t % GT_K; nn = t / GT_K + (256 / GT_K) * j; }
      const int64_t hk = k0 + kn, hn = n0 + nn;
      float w = 0.f;
      if (hk < ke && hn < g.N) w = B_KN ? g.B[hk * g.ldb + hn] : g.B[hn * g.ldb + hk];
      Bs[kn][nn] = w;
    }
    __syncthreads();
    slice_mfma(As, Bs, wm, wn, i, q, acc);
    __syncthreads();
  }
  // D layout: register r of lane (i, q) = C[row 4q + r][col i] of the 16x16 block
#pragma unroll
  for (int bm = 0; bm < WT; ++bm) {
#pragma unroll
    for (int bn = 0; bn < WT; ++bn) {
      const int64_t n = n0 + wn + 16 * bn + i;
      if (n >= g.N) continue;
      const float bias = g.bias ? g.bias[n] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t m = m0 + wm + 16 * bm + 4 * q + r;
        if (m >= g.M) continue;
        float v = acc[bm][bn][r] + bias;
        if (g.relu) v = v > 0.f ? v : 0.f;
        if (g.mask && !(g.mask[m * g.ldm + n] > 0.f)) v = 0.f;
        if (g.atomic) atomicAdd(g.C + m * g.ldc + n, v);
        else g.C[m * g.ldc + n] = v;
      }
    }
  }
}

// emb[p][j] = sin(p.float() @ B)[j] for j < 93, 0 for the pad columns 93..95
__global__ void k_imap_embed(const float4* pf, const float* B, int64_t P, float* emb) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= P * EMBP) return;
  const int64_t p = e / EMBP;
  const int j = (int)(e - p * EMBP);
  float v = 0.f;
  if (j < EMB) {
    const float4 f = pf[p];
    const float x = __builtin_fmaf(f.z, B[2 * EMB + j], __builtin_fmaf(f.y, B[EMB + j], f.x * B[j]));
    v = sinf(x);  // ocml (6.8e-8 abs): |x| <= ~3e2 here; the decoder is 14x the MACs of a NICE MLP
  }
  emb[e] = v;
}

// dx[p][j] = demb[p][j] * cos(x_j) (stored for dB = pf^T dx) and d p.float() = B dx
// -> dpts (float64, the .float() cast's backward).  Block = 2 points x 96 features
// (coalesced row reads), the 3 x 96 products of a point summed through LDS.
constexpr int FB_PTS = 2;
__global__ void __launch_bounds__(FB_PTS * EMBP) k_imap_fourier_bwd(const float4* pf, const float* B, int64_t P,
                                                                     const float* demb, float* dx, double* dpts) {
  __shared__ float red[3][FB_PTS * EMBP];
  const int t = threadIdx.x, lp = t / EMBP, j = t - lp * EMBP;
  const int64_t p = (int64_t)blockIdx.x * FB_PTS + lp;
  float v = 0.f;
  if (p < P && j < EMB) {
    const float4 f = pf[p];
    const float x = __builtin_fmaf(f.z, B[2 * EMB + j], __builtin_fmaf(f.y, B[EMB + j], f.x * B[j]));
    v = demb[p * EMBP + j] * cosf(x);
  }
  if (dx && p < P) dx[p * EMBP + j] = v;  // pad columns 93..95 = 0
  red[0][t] = j < EMB ? B[j] * v : 0.f;
  red[1][t] = j < EMB ? B[EMB + j] * v : 0.f;
  red[2][t] = j < EMB ? B[2 * EMB + j] * v : 0.f;
  __syncthreads();
  if (j < 3 && p < P && dpts) {
    const float* r = red[j] + lp * EMBP;
    float s = 0.f;
    for (int k = 0; k < EMB; ++k) s = s + r[k];
    dpts[p * 3 + j] = (double)s;
  }
}

// out[c] += sum_p X[p*ld + c] (bias gradients).  Block = (up to 64 columns) x (256 / that
// rows) over one point slice; rows summed in LDS, then ONE atomic per column per block
// (same-address atomics serialise in L2: slices, not blocks x rows, set their count).
constexpr int CS_SLICES = 256;
__global__ void __launch_bounds__(256) k_imap_colsum(const float* X, int64_t P, int ld, int ncols, int64_t per,
                                                     float* out) {
  __shared__ float part[256];
  const int cb = ncols < 64 ? ncols : 64, rows = 256 / cb;
  const int cl = threadIdx.x % cb, r = threadIdx.x / cb;
  const int c = blockIdx.x * cb + cl;
  const bool on = r < rows && c < ncols;
  const int64_t pb = (int64_t)blockIdx.y * per;
  const int64_t pe = pb + per < P ? pb + per : P;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // 8 independent loads in flight
  if (on) {
    int64_t p = pb + r;
    for (; p + 7 * rows < pe; p += 8 * rows) {
#pragma unroll
      for (int u = 0; u < 8; ++u) s[u] = s[u] + X[(p + u * rows) * ld + c];
    }
    for (; p < pe; p += rows) s[0] = s[0] + X[p * ld + c];
  }
  part[threadIdx.x] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
  __syncthreads();
  if (r == 0 && c < ncols) {
    float t = 0.f;
    for (int k = 0; k < rows; ++k) t = t + part[k * cb + cl];
    atomicAdd(out + c, t);
  }
}

// raw [P][4] -> occupancy slot / rgb (RayCtx inputs of k_composite_*)
__global__ void k_imap_split(const float* raw, int64_t P, float* occ, float* rgb) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  const float4 r = reinterpret_cast<const float4*>(raw)[p];
  occ[p] = r.w;
  rgb[p * 3 + 0] = r.x;
  rgb[p * 3 + 1] = r.y;
  rgb[p * 3 + 2] = r.z;
}

// d raw [P][4] from k_composite_bwd's (grgb, gocc)
__global__ void k_imap_dout(const float* gocc, const float* grgb, int64_t P, float* dout) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  reinterpret_cast<float4*>(dout)[p] = float4{grgb[p * 3 + 0], grgb[p * 3 + 1], grgb[p * 3 + 2], gocc[p]};
}

// points mode prologue: p.float()
__global__ void k_imap_pf(const double* pts, int64_t P, float4* pf) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  pf[p] = float4{(float)pts[p * 3 + 0], (float)pts[p * 3 + 1], (float)pts[p * 3 + 2], 0.f};
}

static inline unsigned blocks_of(int64_t n, int b) { return (unsigned)((n + b - 1) / b); }

int launch_imap_gemm(const ImapGemm& g, bool a_km, bool b_kn, hipStream_t s) {
  if (g.M <= 0 || g.N <= 0) return 0;
  ImapGemm c = g;
  int splits = 1;
  if (c.atomic && c.K > 0) {  // split the reduction over points so the chip fills
    const int64_t tiles = ((c.M + GT_M - 1) / GT_M) * ((c.N + GT_N - 1) / GT_N);
    const int64_t want = (2048 + tiles - 1) / tiles;
    const int64_t maxs = (c.K + 255) / 256;
    splits = (int)(want < maxs ? want : maxs);
    if (splits < 1) splits = 1;
    if (splits > 65535) splits = 65535;
  }
  c.k_split = ((c.K + splits - 1) / splits + GT_K - 1) / GT_K * GT_K;
  if (c.k_split < GT_K) c.k_split = GT_K;
  splits = (int)((c.K + c.k_split - 1) / c.k_split);
  if (splits < 1) splits = 1;
  const dim3 grid(blocks_of(c.M, GT_M), blocks_of(c.N, GT_N), (unsigned)splits);
  if (!a_km && !b_kn) hipLaunchKernelGGL((k_imap_gemm<false, false>), grid, dim3(256), 0, s, c);
  else if (!a_km && b_kn) hipLaunchKernelGGL((k_imap_gemm<false, true>), grid, dim3(256), 0, s, c);
  else if (a_km && b_kn) hipLaunchKernelGGL((k_imap_gemm<true, true>), grid, dim3(256), 0, s, c);
  else hipLaunchKernelGGL((k_imap_gemm<true, false>), grid, dim3(256), 0, s, c);
  return (int)hipGetLastError();
}

int launch_imap_embed(const float4* pf, const float* B, int64_t P, float* emb, hipStream_t s) {
  if (P <= 0) return 0;
  hipLaunchKernelGGL(k_imap_embed, dim3(blocks_of(P * EMBP, 256)), dim3(256), 0, s, pf, B, P, emb);
  return (int)hipGetLastError();
}

int launch_imap_fourier_bwd(const float4* pf, const float* B, int64_t P, const float* demb, float* dx, double* dpts,
                            hipStream_t s) {
  if (P <= 0) return 0;
  hipLaunchKernelGGL(k_imap_fourier_bwd, dim3(blocks_of(P, FB_PTS)), dim3(FB_PTS * EMBP), 0, s, pf, B, P, demb, dx,
                     dpts);
  return (int)hipGetLastError();
}

int launch_imap_colsum(const float* X, int64_t P, int ld, int ncols, float* out, hipStream_t s) {
  if (P <= 0) return 0;
  if (ncols < 1 || ncols > 256) return (int)hipErrorInvalidValue;
  int64_t slices = (P + 1023) / 1024;
  if (slices > CS_SLICES) slices = CS_SLICES;
  const int64_t per = (P + slices - 1) / slices;
  const int cb = ncols < 64 ? ncols : 64;
  const dim3 grid((unsigned)((ncols + cb - 1) / cb), (unsigned)((P + per - 1) / per));
  hipLaunchKernelGGL(k_imap_colsum, grid, dim3(256), 0, s, X, P, ld, ncols, per, out);
  return (int)hipGetLastError();
}

int launch_imap_split(const float* raw, int64_t P, float* occ, float* rgb, hipStream_t s) {
  if (P <= 0) return 0;
  hipLaunchKernelGGL(k_imap_split, dim3(blocks_of(P, 256)), dim3(256), 0, s, raw, P, occ, rgb);
  return (int)hipGetLastError();
}

int launch_imap_dout(const float* gocc, const float* grgb, int64_t P, float* dout, hipStream_t s) {
  if (P <= 0) return 0;
  hipLaunchKernelGGL(k_imap_dout, dim3(blocks_of(P, 256)), dim3(256), 0, s, gocc, grgb, P, dout);
  return (int)hipGetLastError();
}

int launch_imap_pf(const double* pts, int64_t P, float4* pf, hipStream_t s) {
  if (P <= 0) return 0;
  hipLaunchKernelGGL(k_imap_pf, dim3(blocks_of(P, 256)), dim3(256), 0, s, pts, P, pf);
  return (int)hipGetLastError();
}

}  // namespace nc
