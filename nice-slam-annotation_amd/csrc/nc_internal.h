// nc_internal.h — kernel argument blocks and launch wrappers shared by the
// ABI layer (nc_abi.hip) and the kernels (nc_rays.hip, nc_mlp.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nicecore.h"

namespace nc {

// One decoder evaluation in a stage (decoder.py:341-370): which decoder, its
// output slot, and which gradients the backward must produce for it.
struct Job {
  int32_t kind;        // enum nc_decoder
  int32_t slot;        // index into the per-slot point buffers
  int32_t need_dw;     // decoder parameter gradient
  int32_t need_grid;   // gradient into its own grid (the fine decoder's middle lookup never has one)
  int32_t need_coord;  // gradient into the sample points
  int32_t keep_h;      // forward: store the activation records h_0..h_4 (k_mlp_dw's operands)
  int32_t c_stride;    // floats between consecutive points' features in MlpCtx::cfeat
  int64_t rec_off;     // float offset of this job's point records in MlpCtx::rec
  int64_t c_off;       // float offset of point 0's features in MlpCtx::cfeat
};

constexpr int MAX_JOBS = 3;
// sparse-row claims: wavefront w of a job appends to counter w % CLAIM_SHARDS (one hot
// word saturates near 88 returning atomics per microsecond, MI355X_MICROARCH.md)
constexpr int CLAIM_SHARDS = 64;
static_assert(CLAIM_SHARDS <= 64, "k_rows_compact sums the shard counters across one wavefront");

// Split-f16 forward weight images (nc_wimage.h): extra workgroups of the kernel before
// k_mlp_fwd (k_ray_setup, k_points_prep) build job j's image at img + j * WIMG_STRIDE.
struct WImgCtx {
  int32_t n_jobs;      // 0: no builder workgroups
  int32_t kind[MAX_JOBS];
  int32_t wgs_per_job; // WIMG_WGS (forward image) + WIMG_WGS when dximg is set
  char* img;           // [n_jobs][WIMG_STRIDE] (MlpCtx::wimg)
  float* dximg;        // [n_jobs][DXIMG_STRIDE / 4] k_mlp_dx's f32 image (MlpCtx::dximg), or NULL
  nc_decoder_params dec[MAX_JOBS];
};

// Arguments of the point-batched decoder kernels.
struct MlpCtx {
  int64_t P;                 // number of points
  int32_t n_jobs;
  int32_t slab_wgs;          // workgroups per job in the k_mlp_dw launch (= gridDim.x)
  int32_t save_rec;          // forward: write the activation records
  int32_t share_mid;         // jobs[0] is the fine decoder and jobs[1] the middle one with the
                             // same bound: grid_middle is gathered once for both
  Job jobs[MAX_JOBS];
  nc_grid grids[4];
  nc_decoder_params dec[4];
  const double* pts;         // [P,3] float64 sample points
  const float4* xyz;         // [n_jobs][P] normalize_3d_coordinate(p, decoder bound).float() (w unused)
  const float4* pf;          // [P] p.float() (w unused)
  float* occ;                // [n_jobs][P] occupancy outputs (occupancy decoders)
  float* rgb;                // [P][3] colour-decoder outputs (channels 0..2)
  const float* gocc;         // [P] d loss / d occupancy (shared by the occupancy decoders)
  const float* grgb;         // [P][3] d loss / d rgb
  double* dpts;              // [n_jobs][P][3] per-decoder point gradients
  float* cfeat;              // grid features per job (k_grid_gather -> k_mlp_fwd): the records'
                             // feature field when saving, else a [n_jobs][P][CD] buffer
  float* rec;                // per job [P][Rec::STRIDE]: forward activations (k_mlp_fwd) followed
                             // by backward activations (k_mlp_dx); both read by k_mlp_dw
  float* slab;               // [n_jobs][slab_wgs][slab_stride] per-workgroup parameter gradients
  int64_t slab_stride;
  int32_t fwd_off[MAX_JOBS + 1];  // k_mlp_fwd: workgroups [off[j], off[j+1]) of the 1-D grid run job j
  int32_t dw_off[MAX_JOBS + 1];   // k_mlp_dw: same, and slab row = workgroup index
                                  // (both split in proportion to the decoders' per-point MACs)
  float4* zero_fill;         // optional: k_grid_gather also zero-fills zero_n4 float4s here (the
  int64_t zero_n4;           // caller's gradient buffer, nc_render_args.grad_zero)
  float* jac;                // NC_SAVE_POINT_JACOBIAN: [n_jobs][P][3][32] d own-grid features /
                             // d (ix, iy, iz) (k_grid_gather -> k_mlp_dx), else NULL
  int32_t fuse_gather;       // k_mlp_fwd gathers its tiles' grid features itself (trilinear lookups
                             // of k_grid_gather fused; no claims / Jacobian; zero_fill done by it)
  int32_t claim_rows;        // forward for a backward: k_grid_gather claims sparse gradient rows
                             // (nc_grid.grad_rows) of the grids that have a row map
  int32_t* claim_cnt;        // [MAX_JOBS][CLAIM_SHARDS] claims per shard (zeroed per forward)
  int64_t* claim_tmp;        // [MAX_JOBS][CLAIM_SHARDS][claim_cap] voxels claimed, per shard
  int64_t claim_cap;         // entries per shard: (waves of a job / CLAIM_SHARDS + 1) * 64
  float* dfeat;              // NC_DETERMINISTIC: [n_jobs][P][32] d features of each job's own grid
                             // (k_mlp_dx stores them instead of scattering with atomics), else NULL
  float* bslab;              // [n_jobs][bslab_rows][DX_BSLAB] Fourier-B gradient partials, one row per
  int32_t bslab_rows;        // k_mlp_dx workgroup (= its grid x); k_mlp_dw moves them into its slab
  const double* dout_scale;  // device scalar multiplying gocc / grgb in k_mlp_dx (d loss of a fused
                             // mapper loss, RayCtx::fuse_bwd), or NULL
  const char* wimg;          // [n_jobs][WIMG_STRIDE] split-f16 weight images + flag words (nc_wimage.h),
                             // built by the kernel before k_mlp_fwd (WImgCtx)
  const float* dximg;        // [n_jobs][DXIMG_STRIDE / 4] k_mlp_dx's f32 weight images (Net<KIND, PADW_BWD>),
                             // built with wimg by a forward that saves for the backward
  uint32_t* range_flag;      // [MAX_JOBS] split-f16 range guard: k_mlp_fwd sets job j's word when
                             // an operand reached RANGE_LIMIT, k_mlp_fwd_exact then recomputes the
                             // job in f32; zeroed by k_ray_setup / k_points_prep (NULL: no guard)
};

// NC_DETERMINISTIC grid-gradient scatter (nc_det.hip): every (job, point, corner)
// contribution becomes an entry keyed by (job, voxel); a stable radix sort groups the
// entries of one voxel in ascending (point, corner) order -- the reference's own
// accumulation order (ATen's CPU grid_sampler_3d_backward) -- and one owner per voxel
// sums them in that order.  Run to run bit-identical.
struct DetBufs {
  uint64_t* key[2];          // [n_jobs * ppad * 8] sort keys in / out
  uint32_t* val[2];          // entry ids in / out
  float* w;                  // [n_jobs * ppad * 8] trilinear weight of each entry
  float* part;               // [ceil(entries / (8 DET_DSUB))][2][32] partial sums of the runs that
                             // cross a chunk boundary (k_det_runs -> k_det_join)
  void* temp;                // radix-sort scratch: digit counts per tile + digit totals
  size_t temp_bytes;
  int64_t ppad;              // points per job in the entry arrays: P rounded up to 256 (det_ppad)
  int32_t vbits;             // bits of the voxel index; key = job << vbits | voxel
  int32_t sorted;            // which of key[] / val[] holds the sorted entries (set by the sort)
  int32_t sort_bits;         // radix digit width, fixed with the buffers (det_sort_bits)
};
#ifndef NC_DET_DSUB
#define NC_DET_DSUB 16
#endif
constexpr int DET_DSUB = NC_DET_DSUB;  // entries per k_det_runs sub-chunk (one half-wave; 8 per chunk)
int det_sort_bits(int end_bit);
inline int64_t det_ppad(int64_t P) { return (P + 255) / 256 * 256; }  // one radix tile per 256 points
size_t det_sort_temp_bytes(int64_t n_entries, int bits);
int launch_det_scatter(const MlpCtx& m, const DetBufs& d, hipStream_t s);

// training-ray sampling (nc_sample.hip)
int launch_sample_rays(const nc_sample_args& a, hipStream_t s);
int launch_sample_pose_grad(const nc_sample_args& a, hipStream_t s);
// frustum feature selection (nc_frustum.hip)
int launch_frustum_mask(const nc_frustum_args& a, hipStream_t s);
int launch_grid_rows(const nc_grid_rows_args& a, hipStream_t s);
// importance sampling (nc_pdf.hip)
int launch_sample_pdf(const nc_pdf_args& a, hipStream_t s);
// optimiser step (nc_adam.hip)
int launch_adam(const nc_adam_args& a, hipStream_t s);
int launch_adam_multi(const nc_adam_args& a, const nc_adam_segment* segs, int n, hipStream_t s);
// sparse gradient rows (nc_sparse.hip)
int launch_rows_clear(const nc_sparse_rows& r, hipStream_t s);
int launch_rows_compact(const MlpCtx& m, hipStream_t s);  // after k_grid_gather's claims
size_t rows_merge_temp_bytes(int64_t n_keys, int64_t n_voxels);
int launch_rows_merge(const nc_sparse_rows& in, const nc_sparse_rows& out, const int64_t* all_voxel,
                      const int32_t* all_count, int world, int64_t rank_capacity, void* temp, size_t temp_bytes,
                      hipStream_t s);

// Arguments of the per-ray kernels (sampling, compositing, ray gradients).
struct RayCtx {
  int64_t N;
  int64_t P;
  int32_t S;             // samples per ray
  int32_t n_strat, n_surf;
  int32_t n_extra;       // caller depths merged into the samples (importance pass)
  const double* z_extra; // [N][n_extra]
  double* z_out;         // optional [N][S] sorted sample depths
  float* weights_out;    // optional [N][S] compositing weights
  int32_t stage;
  int32_t occ_a, occ_b;  // occupancy slots summed into raw[...,3] (-1: none)
  int32_t has_rgb;
  int32_t n_jobs;
  const float* rays_o;
  const float* rays_d;
  const float* gt_depth;
  const float* depth_max;  // device scalar (user override or computed into the workspace)
  int32_t dmax_local;      // k_ray_setup reduces max(gt_depth) itself, per workgroup (small N):
                           // no k_depth_max launch
  uint32_t* range_flag;    // [MAX_JOBS] k_mlp_fwd's range flags, zeroed here (MlpCtx::range_flag)
  int32_t lindisp;         // stratified depths linear in disparity (Renderer.py:208-209)
  const float* t_rand;     // [N][n_strat] perturbation draws (Renderer.py:211-219), or NULL
  double bound[3][2];
  float t_strat[NC_MAX_SAMPLES];
  double t_surf[NC_MAX_SURF];
  double* z;             // [N][S]
  double* pts;           // [P][3]
  float4* xyz;           // [n_jobs][P] normalised coordinates per job's decoder bound
  float4* pf;            // [P] p.float()
  double job_bound[MAX_JOBS][3][2];
  const float* occ;      // [n_jobs][P]
  const float* rgb;      // [P][3]
  double* depth;
  double* var;
  float* color;
  const double* g_depth;
  const double* g_var;
  const float* g_color;
  float* gocc;           // [P]
  float* grgb;           // [P][3]
  const double* dpts;    // [n_jobs][P][3]
  float* g_rays_o;
  float* g_rays_d;
  // fused rendering loss (NC_LOSS_*; Mapper.py:603-612, Tracker.py:117-131)
  int32_t loss, loss_flags;
  float w_color;             // float32, as the reference's w * color_loss
  const float* loss_depth;   // [N]
  const float* loss_color;   // [N][3]
  double* loss_out;
  const double* g_loss;
  double* coef_d;            // [N]    d loss / d depth   (k_loss -> k_composite_bwd)
  float* coef_c;             // [N][3] d loss / d colour
  // iMAP* volume density (occupancy: False, common.py:232-247): alpha = 1 - exp(-relu(raw)
  // * dists * ||rays_d||); k_composite_bwd writes d loss / d ||rays_d|| per ray to gnorm,
  // k_ray_grads adds gnorm * rays_d / ||rays_d|| to g_rays_d
  int32_t density;
  float* gnorm;              // [N]
  int32_t fuse_bwd;          // NC_LOSS_MAPPER forward for a backward: k_composite_fwd_loss writes the
                             // loss's d raw for d loss = 1 (gocc / grgb); no k_loss, no k_composite_bwd
  const uint8_t* valid;      // [N] nc_render_args.ray_valid (0 = ray dropped), or NULL
  double* loss_part;         // fused loss: [fused_loss_blocks(N)][2] per-workgroup (depth, colour) sums
  unsigned* loss_count;      // fused loss: workgroups done (zeroed by k_ray_setup; the last one sums)
  // fused loss: the backward's gradient buffer, zero-filled on the CUs the per-ray kernels
  // leave idle: float4s [0, zero_lo4) by zero_wgs_setup extra workgroups of k_ray_setup,
  // [zero_lo4, zero_n4) by zero_wgs extra workgroups of k_composite_fwd_loss
  float4* zero_fill;
  int64_t zero_n4, zero_lo4;
  int32_t zero_wgs, zero_wgs_setup;
};

// k_composite_fwd_loss workgroups for N rays (the length of RayCtx::loss_part)
int64_t fused_loss_blocks(int64_t N);

// ray r is kept (nc_render_args.ray_valid)
// (the flag byte is loaded unconditionally -- from the workspace's sample depths when there
// is no mask -- so the load is not sunk into a branch of its own and waited for alone)
__device__ __forceinline__ bool ray_ok(const RayCtx& c, int64_t r) {
  const uint8_t f = *(c.valid ? c.valid + r : reinterpret_cast<const uint8_t*>(c.z));
  return c.valid == nullptr || f != 0;
}

// One layer GEMM of the iMAP* MLP (nc_imap.hip): C[m][n] (+)= sum_k A(m,k) B(k,n)
struct ImapGemm {
  const float* A;
  const float* B;
  float* C;
  int64_t M, N, K;
  int64_t lda, ldb, ldc;
  const float* bias;   // [N] or NULL
  const float* mask;   // [M][ldm]: output zeroed where mask <= 0 (ReLU backward), or NULL
  int64_t ldm;
  int32_t relu;
  int32_t atomic;      // accumulate with float atomics (split over K)
  int64_t k_split;     // set by the launcher
  // optional pre-split image of B (k_imap_wimage): row n = ceil(K/32) slices of 128 B
  // (hi | lo f16, k_mlp_fwd's swizzled chunk layout); bflag != 0: B reached 2^15
  const unsigned char* Bimg;
  const uint32_t* bflag;
  int64_t bimg_row;    // bytes per image row
};
int launch_imap_gemm(const ImapGemm& g, bool a_kmajor, bool b_kn, hipStream_t s);
struct ImapWImage {  // split-f16 images of up to 4 matrices, B(k, n) = trans ? src[k*ld+n] : src[n*ld+k]
  const float* src[4];
  unsigned char* img[4];   // [N][ceil(K/32)][128 B]
  float* f32t[4];          // optional: B^T as f32 [N][K] (trans only; the exact fallback's copy)
  int32_t N[4], K[4], ld[4], trans[4];
  uint32_t* flag;          // [4], zeroed by the launcher
};
int launch_imap_wimage(const ImapWImage& w, int n, hipStream_t s);
__host__ __device__ inline int64_t imap_wimage_row(int64_t K) { return (K + 31) / 32 * 128; }
int launch_imap_out(const float* h3, const float* wo, const float* bo, int64_t P, float* raw, hipStream_t s);
int launch_imap_out_bwd(const float* dout, const float* wo, const float* h3, int64_t P, float* dz3, hipStream_t s);
int launch_imap_embed(const float4* pf, const float* B, int64_t P, float* emb, hipStream_t s);
int launch_imap_fourier_bwd(const float4* pf, const float* B, int64_t P, const float* demb, float* dx, double* dpts,
                            hipStream_t s);
int launch_imap_colsum(const float* X, int64_t P, int ld, int ncols, float* out, hipStream_t s);
int launch_imap_split(const float* raw, int64_t P, float* occ, float* rgb, hipStream_t s);
int launch_imap_dout(const float* gocc, const float* grgb, int64_t P, float* dout, hipStream_t s);
int launch_imap_pf(const double* pts, int64_t P, float4* pf, hipStream_t s);

struct ParamReduceCtx {
  int32_t n_jobs;
  int32_t slab_wgs;
  int32_t wg_off[MAX_JOBS + 1];  // job j's slab rows [wg_off[j], wg_off[j+1])
  int64_t slab_stride;
  Job jobs[MAX_JOBS];
  float* grad[MAX_JOBS];
  int64_t nparam[MAX_JOBS];
  const float* slab;
};
constexpr int DX_BSLAB = 3 * 96;  // floats per k_mlp_dx workgroup: d B [3][EMBP]

// kernels: launch wrappers (return hipError_t as int)
int launch_depth_max(const float* gt, const uint8_t* valid, int64_t n, float* out, hipStream_t s);
int launch_ray_setup(const RayCtx& c, const WImgCtx& wi, hipStream_t s);
int launch_composite_fwd(const RayCtx& c, hipStream_t s);
int launch_composite_fwd_loss(const RayCtx& c, hipStream_t s);
int launch_composite_bwd(const RayCtx& c, hipStream_t s);
int launch_ray_grads(const RayCtx& c, hipStream_t s);
int launch_loss(const RayCtx& c, hipStream_t s);
int launch_param_reduce(const ParamReduceCtx& c, int64_t max_nparam, hipStream_t s);
int launch_param_ray_reduce(const ParamReduceCtx& c, int64_t max_nparam, const RayCtx& rc, hipStream_t s);
int launch_points_assemble(const MlpCtx& m, int stage, float* raw, hipStream_t s);
int launch_points_split_grad(const MlpCtx& m, int stage, const float* g_raw, float* gocc, float* grgb,
                             hipStream_t s);
int launch_points_grads(const MlpCtx& m, double* g_pts, hipStream_t s);
int launch_points_prep(const MlpCtx& m, const WImgCtx& wi, float4* xyz, float4* pf, hipStream_t s);

int mlp_fwd_lds_bytes();
int mlp_dw_lds_bytes();
int mlp_dx_lds_bytes();
int mlp_blocks_per_cu(int which);  // 0 k_mlp_fwd, 1 k_mlp_dx, 2 k_mlp_dw, 3 k_mlp_fwd (fused gather)
int rec_stride(int kind);  // floats per point of a decoder's [forward | backward] record
int launch_mlp_fwd(const MlpCtx& c, hipStream_t s);  // grid = c.fwd_off[n_jobs]
int decoder_macs(int kind);  // multiply-adds per point of one decoder's forward
int fwd_tile_cost(int kind);  // relative k_mlp_fwd time per tile (split of its workgroups over the jobs)
int launch_mlp_dx(const MlpCtx& c, int grid_x, bool vec, hipStream_t s);  // vec: all job grids channels-last
int launch_mlp_dw(const MlpCtx& c, hipStream_t s);
int launch_grid_gather(const MlpCtx& c, hipStream_t s);
int rec_feat_offset(int kind);  // float offset of the features inside a point record
int64_t max_param_count();

#ifndef NC_FWD_TILES
#define NC_FWD_TILES 1
#endif
#ifndef NC_FWD_THREADS
#define NC_FWD_THREADS 768
#endif
#ifndef NC_FWD_THREADS_FUSED
#define NC_FWD_THREADS_FUSED 768
#endif
constexpr int FWD_TILES = NC_FWD_TILES;      // 16-point tiles per wave sharing the weight fragments
constexpr int FWD_THREADS = NC_FWD_THREADS;  // k_mlp_fwd<false>: waves per workgroup x 64 (157 VGPRs)
// k_mlp_fwd<true> (trilinear lookups fused): 12 waves (3 per SIMD, 168 VGPRs, 6 spills) since its
// lookups gather every corner in one round trip (172 VGPRs at 8 waves; fwd 98.5 -> 89.6 us at C2)
constexpr int FWD_THREADS_FUSED = NC_FWD_THREADS_FUSED;
__host__ __device__ constexpr int fwd_threads(bool fuse) { return fuse ? FWD_THREADS_FUSED : FWD_THREADS; }
#ifndef NC_DX_THREADS
#define NC_DX_THREADS 768
#endif
constexpr int DX_THREADS = NC_DX_THREADS;   // 12 waves x 16 points, barrier-free; 3 waves/SIMD at <= 170 VGPRs
#ifndef NC_DW_THREADS
#define NC_DW_THREADS 1024
#endif
// k_mlp_dw: 16 waves own the dW tiles; 16-point sub-chunks
constexpr int DW_THREADS = NC_DW_THREADS;

}  // namespace nc
