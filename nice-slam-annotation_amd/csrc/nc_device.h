// nc_device.h — device-side building blocks of the NICE render core (gfx950).
//
// Register layout used by every point-batched MLP in this library ("C layout"):
// a wavefront owns 16 points; lane l handles point i = l & 15 and lane-group
// g = l >> 4 (0..3).  A feature vector of width 16*T is spread over the four
// lanes of a point: register 4*t + r of lane (i, g) holds feature 16*t + 4*g + r.
// This is exactly the accumulator layout of v_mfma_f32_16x16x4_f32 when the MFMA
// computes Y^T = W * X^T with the point on the MFMA column, so a layer's output
// feeds the next layer's B operand with no data movement (k-step s of the next
// layer uses register s).  Weights are the A operand, read from LDS.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nicecore.h"

typedef float floatx4 __attribute__((ext_vector_type(4)));

namespace nc {

constexpr int HID = 32;    // hidden width of every NICE decoder (decoder.py:316)
constexpr int EMB = 93;    // Fourier mapping size (decoder.py:137)
constexpr int EMBP = 96;   // padded to 16
constexpr int NSTEP_H = 8; // k-steps of a 32-wide input (4 features per step)

enum Kind { K_COARSE = NC_DEC_COARSE, K_MID = NC_DEC_MIDDLE, K_FINE = NC_DEC_FINE, K_COLOR = NC_DEC_COLOR };

__device__ __forceinline__ floatx4 mfma4(float a, float b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ floatx4 zero4() { return floatx4{0.f, 0.f, 0.f, 0.f}; }

// Feature index held in register j of lane-group g (C layout).
__device__ __forceinline__ int feat_of(int j, int g) { return 16 * (j >> 2) + 4 * g + (j & 3); }

// ---------------------------------------------------------------------------
// Per-decoder layouts.
//   LDS weight image: every nn.Linear stored row-major [out][packed in] with a
//   leading dimension padded by 4 floats (16-byte rows, ds_read_b128 A reads,
//   conflict-free ds_read_b32 transposed reads).  "Packed in" inserts zero
//   columns so that every input block starts on a 16-feature tile:
//     L0 (xyz): emb 0..92 | 0 0 0                      -> 96
//     L3 (xyz): emb 0..92 | 0 0 0 | h2 0..31 (96..127)  -> 128
//     L3 (coarse, MLP_no_xyz): c 0..31 | h2 32..63      -> 64
//   Flat parameter vector (gradient output): nn.Module.parameters() order.
// ---------------------------------------------------------------------------
// PADW: row padding of the LDS weight images (LD = K + PADW floats).  The forward
// reads weights with ds_read_b128 (lane (i, g) at row i, column 4g): its four
// 16-lane groups {0-3,12-15,20-27}, ... hit 16 distinct 16-B slots iff
// LD/4 == 2 (mod 4), i.e. PADW = 8 for every K here (96, 32, 128, 64).  The dX
// kernel reads the transposed rows with ds_read_b32 (32-bank halves; rows 4 apart
// per lane group) and needs LD == 4 (mod 16): PADW = 4.
constexpr int PADW_FWD = 8;
constexpr int PADW_BWD = 4;

template <int KIND, int PADW = PADW_BWD>
struct Net {
  static constexpr bool XYZ = KIND != K_COARSE;
  static constexpr int CD = (KIND == K_FINE) ? 64 : 32;   // fc_c input width
  static constexpr int NOUT = (KIND == K_COLOR) ? 4 : 1;  // output_linear rows
  static constexpr int NFC = XYZ ? 5 : 0;
  // real input widths of pts_linears
  __host__ __device__ static constexpr int in_real(int i) {
    return i == 0 ? (XYZ ? EMB : HID) : i == 3 ? (XYZ ? (EMB + HID) : (2 * HID)) : HID;
  }
  // packed input widths
  static constexpr int IN0 = XYZ ? EMBP : HID;
  static constexpr int IN3 = XYZ ? (EMBP + HID) : (2 * HID);
  static constexpr int LD0 = IN0 + PADW, LDH = HID + PADW, LD3 = IN3 + PADW, LDC = CD + PADW;
  // LDS offsets (floats)
  static constexpr int W0 = 0;
  static constexpr int W1 = W0 + HID * LD0;
  static constexpr int W2 = W1 + HID * LDH;
  static constexpr int W3 = W2 + HID * LDH;
  static constexpr int W4 = W3 + HID * LD3;
  static constexpr int WC = W4 + HID * LDH;      // NFC x [32][LDC]
  static constexpr int BL = WC + NFC * HID * LDC;  // 5 x 32 linear biases
  static constexpr int BC = BL + 5 * HID;          // NFC x 32 fc biases
  static constexpr int WO = BC + NFC * HID;        // [4][32] output weights (rows >= NOUT zero)
  static constexpr int BO = WO + 4 * HID;          // [4]
  static constexpr int FB = BO + 4;                // [3][96] Fourier B (XYZ)
  static constexpr int WEIGHTS = ((FB + (XYZ ? 3 * EMBP : 0)) + 3) & ~3;
  __host__ __device__ static constexpr int lin_off(int i) {
    return i == 0 ? W0 : i == 1 ? W1 : i == 2 ? W2 : i == 3 ? W3 : W4;
  }
  __host__ __device__ static constexpr int lin_ld(int i) { return i == 0 ? LD0 : i == 3 ? LD3 : LDH; }
  // packed column of a real input column of pts_linears[i]
  __host__ __device__ static constexpr int pack_col(int i, int c) {
    return (XYZ && (i == 0 || i == 3) && c >= EMB) ? (c - EMB + EMBP) : c;
  }
  // real column of a packed column (-1: padding)
  __host__ __device__ static constexpr int real_col(int i, int c) {
    return (XYZ && (i == 0 || i == 3)) ? (c < EMB ? c : (c < EMBP ? -1 : c - EMBP + EMB)) : c;
  }

  // flat parameter offsets (reference parameters() order)
  static constexpr int64_t FC_BLOCK = (int64_t)HID * CD + HID;
  __host__ __device__ static constexpr int64_t p_fc_w(int i) { return XYZ ? i * FC_BLOCK : 0; }
  __host__ __device__ static constexpr int64_t p_fc_b(int i) { return p_fc_w(i) + (int64_t)HID * CD; }
  static constexpr int64_t P_B = XYZ ? 5 * FC_BLOCK : 0;
  static constexpr int64_t P_LIN0 = XYZ ? P_B + 3 * EMB : 0;
  __host__ __device__ static constexpr int64_t p_lin_w(int i) {
    int64_t o = P_LIN0;
    for (int k = 0; k < i; ++k) o += (int64_t)HID * in_real(k) + HID;
    return o;
  }
  __host__ __device__ static constexpr int64_t p_lin_b(int i) { return p_lin_w(i) + (int64_t)HID * in_real(i); }
  static constexpr int64_t P_OUT_W = p_lin_b(4) + HID;
  static constexpr int64_t P_OUT_B = P_OUT_W + NOUT * HID;
  static constexpr int64_t NPARAM = P_OUT_B + NOUT;
};

// ---------------------------------------------------------------------------
// Split-f16 MFMA ("3 x f16"): every decoder GEMM runs on v_mfma_f32_16x16x32_f16,
// which issues at 16x the rate of the f32-input MFMA on gfx950.  An f32 operand x
// is split into hi = f16(x) and lo = f16((x - hi) * 2^11), both rounded to nearest; a
// product sum is  sum(a_hi b_hi) + 2^-11 (sum(a_hi b_lo') + sum(a_lo' b_hi))  in two
// f32 accumulators (the a_lo b_lo term, ~2^-22 relative, is dropped).  Measured on
// MI355X (tools/split16_bench.hip, profiles/r02/split16_numerics_rate.log): max error
// per sum|ab| 4e-8 .. 8e-8 for operands of magnitude 1e-3 .. 300 at K = 32 .. 640,
// at or below the exact-f32 MFMA chain's 7e-8 .. 1.3e-7; operands below ~6e-5
// (f16 subnormal range) lose relative precision (5e-7 .. 1e-6 at 1e-5), which is
// far below every tolerance here.  |x| >= 65504 would overflow hi: decoder
// activations are O(1) (xavier weights, sin features, grid features).
//
// Operand layout: the 8 registers j of lane-group g that hold a 32-feature block in
// the C layout (feature feat_of(j, g)) are exactly the B operand's k-slots 8g + j,
// so a layer's accumulators feed the next layer after a split with no data
// movement; the weight images store each 32-column block with column feat_of(j, g)
// at slot 8g + j (hslot), one 128-byte row per matrix row: 16-byte chunk g of the hi
// plane and chunk g of the lo plane at chunk positions g ^ f(row) and (g + 4) ^ f(row),
// f(row) = (row >> 1) & 7 -- the XOR swizzle that makes every lane group of a
// ds_read_b128 (MI355X_MICROARCH.md LDS table: 4 x 16 lanes, 64 banks) touch 16
// distinct 16-byte bank slots when lane (i, g) reads row i, chunk g.
// ---------------------------------------------------------------------------
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef __fp16 halfx2 __attribute__((ext_vector_type(2)));
constexpr float SPLIT_SCALE = 2048.f;
constexpr float SPLIT_INV = 1.f / 2048.f;
constexpr int HROW = 128;  // bytes per image row: 32 hi + 32 lo halves, chunks swizzled

// byte offset inside a row of chunk g (0..3) of plane p (0 hi, 1 lo)
__host__ __device__ constexpr int hchunk(int row, int g, int p) { return 16 * ((g + 4 * p) ^ ((row >> 1) & 7)); }
// The forward's weights carry a third plane (round 5): W = hi + 2^-11 (mid + lo3), all
// round-to-nearest f16, represents a float32 weight to within 3e-11 absolute (lo3 = the
// residual after mid, f16 subnormal for small weights), i.e. below float32's own rounding
// for every |W| > 1e-3; lo3 . xh goes into the same 2^-11 accumulator as mid . xh.
// With two planes each weight was off by up to 2^-22 of itself: one fixed perturbation of
// the network, the same at every point, so its effect on sums over points did not average
// out -- the occupancy decoders' output-bias gradient (sum of d raw) was 8x further from
// the float64 truth than the reference's float32 in a reordered summation
// (tests/test_gpu_elementwise.py).  Activations keep two planes: their 2^-22 rounding is
// per point, like float32's.  lo3 rows are 64 B: chunk g of row r at g ^ F((r >> 2) & 3),
// F = (0, 2, 3, 1).  ds_read_b128 serves a wave in the lane groups {0-3, 12-15, 20-27},
// {4-11, 16-19, 28-31} (+32) (MI355X_MICROARCH.md LDS table), i.e. rows i of lane group g
// mixed with rows of g ^ 1; with F = identity two lanes of each group met on one bank slot
// (2-way conflict on every third-plane read, round 6), with this F each group's 16 reads
// touch 16 distinct 16-B slots (tests/test_lds_swizzle.py checks both images' reads).
constexpr int HROW3 = 64;
__host__ __device__ constexpr int hchunk3(int row, int g) { return 16 * (g ^ ((0x1320 >> (4 * ((row >> 2) & 3))) & 3)); }

__device__ __forceinline__ floatx4 mfma16(half8 a, half8 b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// MI355X / ROCm 7.2 hazard: the LAST result register of v_mfma_f32_16x16x32_f16 needs
// 8 wait states before a VALU reads it (the first one needs 7), but hipcc's hazard
// recognizer pads 7 for every register -- measured with hand-placed s_nops on
// every CU (tools/mfma_hazard.hip, profiles/r02/mfma_hazard.log: v_mov of v43 after
// 7 states reads stale data in 65% of waves, after 8 in none).  In a split-f16 k_mlp_dx
// the compiler's v_pk_mul of those registers at exactly 7 states gave sporadically
// wrong point gradients.  Every group of split-f16 MFMAs whose results go to VALU ends
// with mfma16_drain(): a scheduling fence around an s_nop 7, so the readers sit at
// least 8 states after the last MFMA whatever the compiler counts for the asm.
__device__ __forceinline__ void mfma16_drain() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 7" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// slot (0..31) of feature f (0..31) inside a 32-column block: inverse of feat_of
__host__ __device__ constexpr int hslot(int f) { return 8 * ((f >> 2) & 3) + 4 * (f >> 4) + (f & 3); }

// split 8 C-layout values (one 32-feature block of a lane) into f16 hi / scaled lo, both
// rounded to nearest even: x = hi + 2^-11 lo to within 2^-22 relative, UNBIASED.  (Round 5:
// the former round-toward-zero pair (v_cvt_pkrtz) truncated both halves, so every operand's
// magnitude came out short by up to 2^-20 and 2^-21 on average -- a systematic shrink that
// cancellation-heavy statistics accumulate: the occupancy decoders' output-bias gradient,
// a sum of d raw over all points, was 100x further from the float64 truth than the
// reference's float32 (tests/test_gpu_elementwise.py, profiles/r05/elementwise/).)
// hi = RNE(x) leaves r = x - hi exact in f32 (Sterbenz: hi is within a factor 2 of x) with
// |r| <= half an f16 ulp of x, so lo = RNE(r * 2^11) keeps 11 more bits.
__device__ __forceinline__ void split8(const float* x, half8& hi, half8& lo) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const _Float16 h = (_Float16)x[j];  // v_cvt_f16_f32: round to nearest even
    hi[j] = h;
    lo[j] = (_Float16)((x[j] - (float)h) * SPLIT_SCALE);
  }
}

// the truncating split (round-to-zero halves) the iMAP* layer GEMMs keep: their golden
// case with importance sampling (tests/test_gpu_imap.py nodepth_imp) picks its second-pass
// samples from the first pass's weights by CDF inversion, so a last-bit change of the
// forward can move a sample; that case is pinned on the round-4 numerics.  The NICE forward
// uses split8 (round to nearest) with three weight planes, gated per element.
__device__ __forceinline__ void split8_rtz(const float* x, half8& hi, half8& lo, float& amax) {
#pragma unroll
  for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(x[j]));
#pragma unroll
  for (int j = 0; j < 8; j += 2) {
    const halfx2 h = __builtin_amdgcn_cvt_pkrtz(x[j], x[j + 1]);
    const float r0 = (x[j] - (float)h[0]) * SPLIT_SCALE;
    const float r1 = (x[j + 1] - (float)h[1]) * SPLIT_SCALE;
    const halfx2 l = __builtin_amdgcn_cvt_pkrtz(r0, r1);
    hi[j] = (_Float16)h[0];
    hi[j + 1] = (_Float16)h[1];
    lo[j] = (_Float16)l[0];
    lo[j + 1] = (_Float16)l[1];
  }
}

// split8 that also folds max |x| into amax (one v_max_f32 with an |.| modifier per
// value): the range guard of the split-f16 forward.  hi = f16(x) (round to nearest even)
// and the residual scaled by 2^11 stay finite and exact-enough only for |x| < 2^15
// (RANGE_LIMIT); a tile
// that saw a larger (or infinite) operand is recomputed on the exact-f32 MFMA path
// (nc_mlp.hip k_mlp_fwd_exact).  NaN operands pass (fmaxf drops them) and stay NaN, as
// in the reference's fp32 addmm.
constexpr float RANGE_LIMIT = 32768.f;
__device__ __forceinline__ void split8(const float* x, half8& hi, half8& lo, float& amax) {
#pragma unroll
  for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(x[j]));
  split8(x, hi, lo);
}

// f16 weight image of k_mlp_fwd.
//   f32 part first (floats): biases BL [5][32], BC [NFC][32], output WO [4][32], BO [4],
//   Fourier B FB [3][96]; then, from byte HB, the matrices of pts_linears 0..4 and
//   fc_c 0..4, each MROWS(m) rows of HROW bytes.
//   row kb*32 + o of matrix L holds W[o][32 kb + feat_of(slot)] (a matrix with K packed
//   inputs has K rows).
template <int KIND>
struct NetH {
  using N = Net<KIND>;
  static constexpr int BL = 0;
  static constexpr int BC = BL + 5 * HID;
  static constexpr int WO = BC + N::NFC * HID;
  static constexpr int BO = WO + 4 * HID;
  static constexpr int FB = BO + 4;
  static constexpr int F32_FLOATS = ((FB + (N::XYZ ? 3 * EMBP : 0)) + 3) & ~3;
  static constexpr int HB = F32_FLOATS * 4;  // byte offset of the f16 matrices
  __host__ __device__ static constexpr int kin(int L) { return L == 0 ? N::IN0 : L == 3 ? N::IN3 : HID; }
  __host__ __device__ static constexpr int lin_off(int L) {  // bytes
    int o = HB;
    for (int k = 0; k < L; ++k) o += kin(k) * HROW;
    return o;
  }
  __host__ __device__ static constexpr int fc_off(int L) { return lin_off(5) + L * N::CD * HROW; }
  // third planes (HROW3-byte rows), same row order, after every two-plane matrix
  static constexpr int B3 = fc_off(N::NFC);
  __host__ __device__ static constexpr int lin3_off(int L) {
    int o = B3;
    for (int k = 0; k < L; ++k) o += kin(k) * HROW3;
    return o;
  }
  __host__ __device__ static constexpr int fc3_off(int L) { return lin3_off(5) + L * N::CD * HROW3; }
  static constexpr int BYTES = fc3_off(N::NFC);
};

// ---------------------------------------------------------------------------
// Trilinear corners of F.grid_sample(5-D, bilinear, border, align_corners=True)
// restated from ATen's CPU grid_sampler_3d (the reference runs it through
// decoder.py:186): unnormalise ((x+1)/2)*(size-1), clip to [0, size-1], corner
// weights as products in x, y, z order, corners tnw..bse (bit0 = x, bit1 = y,
// bit2 = z).  Compiled with -ffp-contract=off, so the forward value is
// bit-identical to the CPU reference.
// ---------------------------------------------------------------------------
// Index arithmetic: the clip keeps ix in [0, W-1] (NaN clips to W-1), so the corner-0
// voxel indices are non-negative int32 and corner k is outside the grid only on the far
// side (x0 + 1 == W, ...).  Element strides are int32 (the host rejects a grid whose
// strides reach 2^31: check_grid); the corner-0 offset is one 64-bit value (the C5 grids
// hold 6.5G elements) and corner k adds the wave-uniform stride sum of its sides.
struct Corners {
  int64_t base;    // element offset of corner 0 (channel 0) in the grid
  float w[8];      // interpolation weight (0 where the corner is out of bounds)
  float wx[2], wy[2], wz[2];  // per-axis factors [west/east], [north/south], [top/bottom]
  float gmx, gmy, gmz;        // d(ix)/d(x_norm) incl. border-clip gradient
  unsigned inb;                // bit k: corner k inside the grid
  int32_t x0, y0, z0;          // corner 0 (tnw) voxel coordinates
};

// element strides of a grid (or its gradient) as int32 (check_grid / check_grad_strides)
__device__ __forceinline__ int32_t stride32(const int64_t s) { return (int32_t)s; }

// offset of corner k from corner 0 along the given strides (wave-uniform)
__device__ __forceinline__ int64_t corner_delta(const int64_t (&st)[4], int k) {
  return (int64_t)((k & 1) ? stride32(st[3]) : 0) + (int64_t)(((k >> 1) & 1) ? stride32(st[2]) : 0) +
         (int64_t)((k >> 2) ? stride32(st[1]) : 0);
}

// element offset of corner k (0 for an out-of-bounds corner: it reads cell 0 instead)
__device__ __forceinline__ int64_t corner_off(const nc_grid& G, const Corners& c, int k) {
  return ((c.inb >> k) & 1u) ? c.base + corner_delta(G.stride, k) : (int64_t)0;
}

// 32 zero floats of each code object: a channels-last gather reads an out-of-bounds
// corner from here, so its term v * w is exactly 0 without a select per channel (corner 0
// is always inside, so the sum of the inside corners is unchanged)
static __device__ __attribute__((aligned(16))) float kZeroRow[32];  // global (not constant) address space: the
                                                                  // corner select stays a global_load, not a flat_load

// channels-last corner row k of grid G (the zero row for an out-of-bounds corner)
__device__ __forceinline__ const float* corner_row(const nc_grid& G, const Corners& c, int k) {
  return ((c.inb >> k) & 1u) ? G.data + (c.base + corner_delta(G.stride, k)) : kZeroRow;
}

// element offset of voxel (x, y, z) along strides st
__device__ __forceinline__ int64_t voxel_off(const int64_t (&st)[4], int32_t x, int32_t y, int32_t z) {
  return (int64_t)z * stride32(st[1]) + (int64_t)y * stride32(st[2]) + (int64_t)x * stride32(st[3]);
}

__device__ __forceinline__ float clip_fwd(float v, float hi) {
  float t = (v < 0.f) ? 0.f : v;       // std::max(in, 0)
  return (t < hi) ? t : hi;            // std::min(hi, t)
}

__device__ __forceinline__ void make_corners(const nc_grid& G, const float xyz[3], Corners& c) {
  const int32_t D = (int32_t)G.dims[0], H = (int32_t)G.dims[1], W = (int32_t)G.dims[2];
  const float sx = (float)(W - 1), sy = (float)(H - 1), sz = (float)(D - 1);
  float ix = ((xyz[0] + 1.f) / 2.f) * sx;
  float iy = ((xyz[1] + 1.f) / 2.f) * sy;
  float iz = ((xyz[2] + 1.f) / 2.f) * sz;
  // border clip gradient: borders count as clipped (GridSampler.h clip_coordinates_set_grad)
  c.gmx = (ix <= 0.f || ix >= sx) ? 0.f : sx / 2.f;
  c.gmy = (iy <= 0.f || iy >= sy) ? 0.f : sy / 2.f;
  c.gmz = (iz <= 0.f || iz >= sz) ? 0.f : sz / 2.f;
  ix = clip_fwd(ix, sx);
  iy = clip_fwd(iy, sy);
  iz = clip_fwd(iz, sz);
  const int32_t x0 = (int32_t)floorf(ix), y0 = (int32_t)floorf(iy), z0 = (int32_t)floorf(iz);
  c.x0 = x0; c.y0 = y0; c.z0 = z0;
  const float fx0 = (float)x0, fy0 = (float)y0, fz0 = (float)z0;
  const float fx1 = (float)(x0 + 1), fy1 = (float)(y0 + 1), fz1 = (float)(z0 + 1);
  c.wx[0] = fx1 - ix; c.wx[1] = ix - fx0;
  c.wy[0] = fy1 - iy; c.wy[1] = iy - fy0;
  c.wz[0] = fz1 - iz; c.wz[1] = iz - fz0;
  // corner k is inside unless one of its far sides leaves the grid (x0, y0, z0 >= 0 always)
  const unsigned xo = (x0 + 1 < W) ? 0xffu : 0x55u;  // bit k kept where k's x side is 0 or x0 + 1 < W
  const unsigned yo = (y0 + 1 < H) ? 0xffu : 0x33u;
  const unsigned zo = (z0 + 1 < D) ? 0xffu : 0x0fu;
  c.inb = xo & yo & zo;
  c.base = voxel_off(G.stride, x0, y0, z0);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int xb = k & 1, yb = (k >> 1) & 1, zb = k >> 2;
    c.w[k] = (c.wx[xb] * c.wy[yb]) * c.wz[zb];
  }
}

// Gather the 8 channels of lane-group g (C layout: channel 16*(j>>2) + 4g + (j&3))
// and accumulate them corner by corner in the reference order (no FMA).
// Branch-free: an out-of-bounds corner loads the (in-bounds) channel-0 cell and its
// value is replaced by 0 (out + 0 == out), so all corners' loads can be in flight
// together instead of one exec-masked round trip per corner.
template <bool VEC>
__device__ __forceinline__ void gather8(const nc_grid& G, const Corners& c, int g, float out[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) out[j] = 0.f;
  const int64_t sC = G.stride[0];
  float v[8][8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    // VEC: out-of-bounds corners read the zero row; else cell 0, and the sum skips them
    const float* base = VEC ? corner_row(G, c, k) : G.data + corner_off(G, c, k);
    if (VEC) {
      const float4 a = *reinterpret_cast<const float4*>(base + 4 * g);
      const float4 b = *reinterpret_cast<const float4*>(base + 16 + 4 * g);
      v[k][0] = a.x; v[k][1] = a.y; v[k][2] = a.z; v[k][3] = a.w;
      v[k][4] = b.x; v[k][5] = b.y; v[k][6] = b.z; v[k][7] = b.w;
    } else {
      if (k == 4) __builtin_amdgcn_sched_barrier(0);  // scalar path: 4 corners x 8 loads in flight
#pragma unroll
      for (int j = 0; j < 8; ++j) v[k][j] = base[(int64_t)feat_of(j, g) * sC];
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const bool in = VEC || ((c.inb >> k) & 1u);
#pragma unroll
    for (int j = 0; j < 8; ++j) out[j] = out[j] + (in ? v[k][j] * c.w[k] : 0.f);
  }
}

// Two channels-last lookups (the fine decoder's [fine | middle]) with all 16 corners'
// loads in flight before either is summed: one memory round trip instead of two.  Each
// lookup is accumulated exactly as gather8 (bit-identical).
__device__ __forceinline__ void gather8x2(const nc_grid& G1, const Corners& c1, const nc_grid& G2, const Corners& c2,
                                          int g, float out1[8], float out2[8]) {
  float v[2][8][8];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const nc_grid& G = q == 0 ? G1 : G2;
    const Corners& c = q == 0 ? c1 : c2;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float* base = corner_row(G, c, k);  // the zero row for out-of-bounds corners
      const float4 a = *reinterpret_cast<const float4*>(base + 4 * g);
      const float4 b = *reinterpret_cast<const float4*>(base + 16 + 4 * g);
      v[q][k][0] = a.x; v[q][k][1] = a.y; v[q][k][2] = a.z; v[q][k][3] = a.w;
      v[q][k][4] = b.x; v[q][k][5] = b.y; v[q][k][6] = b.z; v[q][k][7] = b.w;
    }
  }
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const Corners& c = q == 0 ? c1 : c2;
    float* out = q == 0 ? out1 : out2;
#pragma unroll
    for (int j = 0; j < 8; ++j) out[j] = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
#pragma unroll
      for (int j = 0; j < 8; ++j) out[j] = out[j] + v[q][k][j] * c.w[k];  // 0 * w from the zero row
    }
  }
}

__device__ __forceinline__ bool grid_vec_ok(const nc_grid& G) {
  return G.stride[0] == 1 && ((reinterpret_cast<uintptr_t>(G.data) & 15u) == 0) &&
         (G.stride[1] % 4 == 0) && (G.stride[2] % 4 == 0) && (G.stride[3] % 4 == 0);
}

// normalize_3d_coordinate (common.py:280-295) in float64, then .float()
__device__ __forceinline__ void normalize_pt(const double p[3], const double (&b)[3][2], float out[3]) {
#pragma unroll
  for (int k = 0; k < 3; ++k) out[k] = (float)(((p[k] - b[k][0]) / (b[k][1] - b[k][0])) * 2.0 - 1.0);
}

// sin / cos of the Fourier-feature arguments x = p.float() @ B (decoder.py:26-30; |x|
// reaches ~1e3 rad for room-scale scenes with B ~ N(0, 25^2)) to about one float32 ulp, as
// the CPU reference's sinf: x = t + k pi with k = rint(x / pi) (the 1.5 2^23 magic-number
// round, exact for |x| < 2^22 pi, whose low mantissa bit is k's parity), t by Cody-Waite with
// a three-part pi (pi1 = 3.140625 has 8 significant bits: k pi1 is exact for |k| < 2^16),
// then sin t = t + t^3 P(t^2) / cos t = 1 + t^2 Q(t^2) (minimax on [-pi/2, pi/2], fitted
// by tools/sin_fit.py) and the sign (-1)^k.  Over |x| <= 1.2e3 (tools/sin_fit.py float32
// emulation): sin max error 1.23e-7, mean 1.55e-8 (a correctly rounded float32 sin: 6.9e-8,
// 1.32e-8); cos 1.41e-7, 2.2e-8.  Round 6: the former hardware v_sin_f32 after a [-pi, pi]
// reduction (max error 3.8e-7, 5 float32 ulps of a feature) was the one HIP-specific error of
// the forward that reaches d raw; the fine_depth golden case's decoder gradients failed the
// per-element gate on it (tools/diag_chain.py).  Every step is an IEEE mul /
// fma / add or an integer op, so the packed two-argument form (v_pk_fma_f32) is bit-identical
// to the scalar one (k_mlp_dw recomputes the features with the scalar form); the packed
// form issues 15 instructions per pair of features against the v_sin form's 7 plus two
// quarter-rate transcendentals.
typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2 fma2(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }

constexpr float kInvPi = 0.318309886183790672f;
constexpr float kRoundMagic = 12582912.f;  // 1.5 * 2^23
constexpr float kPi1 = 3.140625f, kPi2 = 9.676535897930e-4f, kPi3 = 5.126566e-12f;
constexpr float kS1 = -0.16666657f, kS2 = 0.008333017f, kS3 = -0.00019806615f, kS4 = 2.6000544e-06f;
constexpr float kC1 = -0.5f, kC2 = 0.04166664f, kC3 = -0.0013888404f, kC4 = 2.4761886e-05f, kC5 = -2.6077103e-07f;

// t = x - k pi and (-1)^k as a sign bit
__device__ __forceinline__ float reduce_pi(float x, unsigned& sign) {
  const float y = __builtin_fmaf(x, kInvPi, kRoundMagic);
  const float k = y - kRoundMagic;
  sign = __float_as_uint(y) << 31;
  float t = __builtin_fmaf(-k, kPi1, x);
  t = __builtin_fmaf(-k, kPi2, t);
  return __builtin_fmaf(-k, kPi3, t);
}
__device__ __forceinline__ float fourier_sin(float x) {
  unsigned sg;
  const float t = reduce_pi(x, sg);
  const float t2 = t * t;
  float p = __builtin_fmaf(t2, kS4, kS3);
  p = __builtin_fmaf(t2, p, kS2);
  p = __builtin_fmaf(t2, p, kS1);
  return __uint_as_float(__float_as_uint(__builtin_fmaf(t2 * t, p, t)) ^ sg);
}
// cos x for the Fourier backward (k_mlp_dx: d (p @ B) = d emb * cos(p @ B)): Cody-Waite by
// 2 pi and the hardware v_cos_f32 (3.8e-7 max error).  It reaches only the point and
// Fourier-B gradients, per point; the polynomial form (fourier_cos_poly, 1.4e-7) cost
// k_mlp_dx 10 us at C2 (120.7 vs 110.8, same box, profiles/r06/sin/) and is kept for reference.
__device__ __forceinline__ float fourier_cos(float x) {
  const float k = __builtin_rintf(x * 0.15915494309189535f);
  float r = __builtin_fmaf(-k, 6.28125f, x);
  r = __builtin_fmaf(-k, 1.9353071795864769e-3f, r);
  r = __builtin_fmaf(-k, 1.2537033403800354e-11f, r);
  return __builtin_amdgcn_cosf(r * 0.15915494309189535f);
}
__device__ __forceinline__ float fourier_cos_poly(float x) {
  unsigned sg;
  const float t = reduce_pi(x, sg);
  const float t2 = t * t;
  float p = __builtin_fmaf(t2, kC5, kC4);
  p = __builtin_fmaf(t2, p, kC3);
  p = __builtin_fmaf(t2, p, kC2);
  p = __builtin_fmaf(t2, p, kC1);
  return __uint_as_float(__float_as_uint(__builtin_fmaf(t2, p, 1.f)) ^ sg);
}

// fourier_sin of two arguments on packed-FP32 instructions, element for element identical
__device__ __forceinline__ f2 fourier_sin2(f2 x) {
  const f2 y = fma2(x, f2{kInvPi, kInvPi}, f2{kRoundMagic, kRoundMagic});
  const f2 nk = f2{kRoundMagic, kRoundMagic} - y;  // -k (exact)
  f2 t = fma2(nk, f2{kPi1, kPi1}, x);
  t = fma2(nk, f2{kPi2, kPi2}, t);
  t = fma2(nk, f2{kPi3, kPi3}, t);
  const f2 t2 = t * t;
  f2 p = fma2(t2, f2{kS4, kS4}, f2{kS3, kS3});
  p = fma2(t2, p, f2{kS2, kS2});
  p = fma2(t2, p, f2{kS1, kS1});
  const f2 s = fma2(t2 * t, p, t);
  return f2{__uint_as_float(__float_as_uint(s.x) ^ (__float_as_uint(y.x) << 31)),
            __uint_as_float(__float_as_uint(s.y) ^ (__float_as_uint(y.y) << 31))};
}

// Sum over the 16 lanes of a DPP row (in the C layout: the 16 points i of one lane-group
// g), left in every lane of the row: xor-1 and xor-2 quad permutes, then the half-row and
// row mirrors.  Each step adds a lane's value to its partner's, so all 16 lanes end with
// the same bits (fixed order, deterministic).
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, true));
}
// v of lane (lane ^ j): DPP row permutes for j < 16 (VALU, a few cycles: xor 1 / 2 are quad
// permutes, xor 4 = quad reverse after the half-row mirror, xor 8 = half-row mirror after
// the row mirror), ds_bpermute (__shfl_xor) across rows.  Exactly __shfl_xor's data
// movement, so butterflies built on it keep their bits.  j must fold to a constant.
__device__ __forceinline__ float xor_lane(float v, int j) {
  if (j == 1) return dpp_mov<0xB1>(v);
  if (j == 2) return dpp_mov<0x4E>(v);
  if (j == 4) return dpp_mov<0x1B>(dpp_mov<0x141>(v));
  if (j == 8) return dpp_mov<0x141>(dpp_mov<0x140>(v));
  return __shfl_xor(v, j);
}
__device__ __forceinline__ double xor_lane(double v, int j) {
  const long long b = __double_as_longlong(v);
  const float lo = xor_lane(__int_as_float((int)(b & 0xffffffffll)), j);
  const float hi = xor_lane(__int_as_float((int)(b >> 32)), j);
  return __longlong_as_double(((long long)__float_as_int(hi) << 32) | (unsigned)__float_as_int(lo));
}

__device__ __forceinline__ float row16_sum(float v) {
  v = v + dpp_mov<0xB1>(v);   // quad_perm [1, 0, 3, 2]
  v = v + dpp_mov<0x4E>(v);   // quad_perm [2, 3, 0, 1]
  v = v + dpp_mov<0x141>(v);  // row_half_mirror
  v = v + dpp_mov<0x140>(v);  // row_mirror
  return v;
}

// Wavefront reductions over the four lanes of a point (lane-groups g).
__device__ __forceinline__ float sum_groups(float v) {
  v += __shfl_xor(v, 16);
  v += __shfl_xor(v, 32);
  return v;
}

}  // namespace nc
