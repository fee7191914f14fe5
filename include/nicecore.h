/*
 * nicecore.h — C ABI of libnicecore.so, the MI355X (gfx950) render core for
 * NICE-SLAM's hot path.
 *
 * What each entry point replaces in the reference (WohimLee/NICE-SLAM-annotation):
 *
 *   nc_render_forward   src/utils/Renderer.py:95-262  Renderer.render_batch_ray forward:
 *                       near/far + bbox (:120-159), surface samples (:162-200),
 *                       stratified samples (:203-219), merge-sort (:222-224),
 *                       points (:227-231), eval_points (:36-93) -> NICE.forward
 *                       (src/conv_onet/models/decoder.py:336-370, MLP :190-219,
 *                       MLP_no_xyz :285-297, grid_sample :179-188), and
 *                       raw2outputs_nerf_color (src/common.py:215-256).
 *   nc_render_backward  autograd backward of the same graph: d/d rays_o, rays_d,
 *                       the four feature grids and every decoder parameter.
 *   nc_points_forward   src/conv_onet/models/decoder.py:336-370 NICE.forward on
 *   nc_points_backward  caller-given points (Renderer.eval_points / Mesher use).
 *   nc_sample_rays_*    src/common.py:74-137 get_samples / get_rays_from_uv over a
 *                       batch of frames + the Tracker/Mapper bbox pre-filter, and the
 *                       pose gradient (Tracker.py:95-111, Mapper.py:543-591).
 *   nc_frustum_mask     src/Mapper.py:100-187 get_mask_from_c2w (frustum feature
 *                       selection of one grid).
 *   nc_adam_step        torch.optim.Adam / SparseAdam step (src/Mapper.py:462-485, :625)
 *   nc_sample_pdf       src/common.py:19-63 sample_pdf (importance sampling,
 *                       Renderer.py:244-250 when N_importance > 0).
 *   nc_sparse_rows_*    the touched-voxel gradient of a feature grid too large for a
 *                       dense gradient: the reference's dense
 *                       grid.grad / val[mask] gradient (Mapper.py:392-404, :620-627)
 *                       restricted to the voxels the batch touched, and its
 *                       multi-rank union before the RCCL sum.
 *
 * Conventions
 *   - All pointers are device pointers on the current HIP device; the library
 *     never allocates or frees device memory.  Scratch state lives in a caller-
 *     allocated workspace of nc_*_workspace_bytes() bytes that must be passed,
 *     unchanged, to the matching backward call.
 *   - Work is enqueued on `stream` (a hipStream_t passed as void*); no call
 *     synchronises the host, so the calls are graph-capturable.
 *   - Return value 0 = success; negative = error (message via nc_last_error(),
 *     thread-local).  No exception crosses this boundary.
 *   - A backward call needs the forward to have run with NC_SAVE_FOR_BACKWARD in
 *     `flags` (the forward then keeps each decoder's per-point activations in the
 *     workspace; the flag also sizes the workspace).  Forward-only callers leave it
 *     0 and get a much smaller workspace.
 *   - Gradient outputs are ACCUMULATED into for grids (caller zero-fills them) and
 *     OVERWRITTEN for rays and decoder parameters.
 */
#ifndef NICECORE_H
#define NICECORE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NC_ABI_VERSION 11
#define NC_MAX_SAMPLES 64 /* n_strat + n_surf per ray (one wavefront per ray) */
#define NC_MAX_SURF 32

/* nc_*_args.flags */
#define NC_SAVE_FOR_BACKWARD 1
/* Grid gradients by an ordered reduction instead of float atomics: bit-identical run
 * to run, summed per voxel in the reference's order (ascending point, corner).  Set it
 * on the forward (it sizes the workspace) and keep it for the backward. */
#define NC_DETERMINISTIC 2
/* The backward will ask for ray / point gradients (ABI v5): the forward then also keeps
 * each decoder lookup's trilinear Jacobian d features / d (ix, iy, iz) (3 x 32 floats
 * per point, from the corner values it gathers anyway), and the backward's coordinate
 * gradient is 96 multiply-adds per point instead of 8 corner re-reads.  Without it a
 * backward with g_rays_* / g_pts re-reads the corners. */
#define NC_SAVE_POINT_JACOBIAN 4
/* nc_render_backward only (ABI v7): stop after the grid and ray gradients; the decoder
 * weight gradients (k_mlp_dw + slab reduction) are left to nc_render_backward_params,
 * called later on the same workspace.  Lets a data-parallel caller start the grid-
 * gradient all-reduce while the weight gradients are still being computed. */
#define NC_DEFER_PARAM_GRADS 8
/* nc_render_forward / _backward (ABI v8, additive): the backward will not ask for decoder
 * `kind`'s weight gradient (its parameters do not require grad: the Tracker's frozen
 * decoders, the Mapper's fix_fine).  The forward then skips that decoder's per-point
 * activation records (5 x 32 floats per point), which only k_mlp_dw reads; a backward
 * that asks for the weight gradient anyway fails.  Keep the same flags on both calls. */
#define NC_NO_WEIGHT_GRAD(kind) (16 << (kind))
#define NC_NO_WEIGHT_GRAD_ALL (16 | 32 | 64 | 128)

/* nc_render_args.loss: the rendering loss computed by the core (optional) */
#define NC_LOSS_NONE 0
#define NC_LOSS_MAPPER 1  /* src/Mapper.py:603-612: sum_{gt>0} |gt - depth| [+ w * sum |gt_color - color|] */
#define NC_LOSS_TRACKER 2 /* src/Tracker.py:117-131: sum_mask |gt - depth| / sqrt(unc + 1e-10) [+ w * color] */
/* nc_render_args.loss_flags */
#define NC_LOSS_COLOR 1   /* add the colour term (Mapper: stage 'color'; Tracker: use_color_in_tracking) */
#define NC_LOSS_DYNAMIC 2 /* Tracker handle_dynamic: mask &= tmp < 10 * median(tmp) (<= 16384 rays) */

/* Stage names of render_batch_ray / NICE.forward (decoder.py:341-370). */
enum nc_stage { NC_STAGE_COARSE = 0, NC_STAGE_MIDDLE = 1, NC_STAGE_FINE = 2, NC_STAGE_COLOR = 3 };

/* Decoders of NICE (decoder.py:321-334) and the grid each one samples. */
enum nc_decoder { NC_DEC_COARSE = 0, NC_DEC_MIDDLE = 1, NC_DEC_FINE = 2, NC_DEC_COLOR = 3 };

/* One feature grid c['grid_*'], shape [1, 32, D, H, W] float32 (NICE_SLAM.py:243-320).
 * Strides are in elements for the C, D, H, W axes; channel stride 1
 * (torch.channels_last_3d) is the fast path.
 *
 * Sparse gradient rows (ABI v5, optional; grad_rows != NULL): instead of a dense
 * [1,32,D,H,W] gradient, `grad` is a compact [row_capacity][32] float buffer (row
 * stride 32, channel stride 1; grad_stride is ignored) holding one row per touched
 * voxel.  grad_rows is a [D*H*W] int32 map voxel (z*H + y)*W + x -> row, -1 where
 * the voxel has no row (all -1 the first time; nc_sparse_rows_clear restores that).
 * A forward with NC_SAVE_FOR_BACKWARD claims a row for every in-bounds corner of
 * every lookup that will receive a grid gradient (first come, first served: the row
 * order is not deterministic), zero-fills it and records its voxel in row_voxel;
 * *row_count counts the rows.  Claims accumulate over forwards until cleared, so
 * several forwards may precede one backward.  row_capacity >= 8 x the lookups of
 * the batch (or D*H*W) never overflows; an overflowing claim is dropped and flagged
 * by *row_count > row_capacity.  The backward accumulates into the rows. */
typedef struct nc_grid {
  const float* data;
  float* grad;            /* NULL: no gradient wanted for this grid */
  int64_t dims[3];        /* D, H, W */
  int64_t stride[4];      /* C, D, H, W strides of data */
  int64_t grad_stride[4]; /* C, D, H, W strides of grad */
  int32_t* grad_rows;     /* sparse mode: [D*H*W] voxel -> gradient row, or NULL (dense) */
  int64_t* row_voxel;     /* [row_capacity] voxel of each row */
  int32_t* row_count;     /* device counter of claimed rows */
  int64_t row_capacity;
} nc_grid;

/* Parameters of one decoder, pointers to the nn.Parameter storage (contiguous,
 * nn.Linear [out,in] row-major).  MLP (decoder.py:116-177): fc_c[5], embedder._B,
 * pts_linears[5], output_linear.  MLP_no_xyz (decoder.py:239-271): pts_linears[5],
 * output_linear (fc_w/fc_b/fourier_B unused). */
typedef struct nc_decoder_params {
  const float* fc_w[5];
  const float* fc_b[5];
  const float* fourier_B; /* [3, 93] */
  const float* lin_w[5];
  const float* lin_b[5];
  const float* out_w;
  const float* out_b;
  float* grad;            /* flat gradient in nn.Module.parameters() order, or NULL */
  double bound[3][2];     /* the decoder's own .bound (coarse: bound * coarse_bound_enlarge) */
} nc_decoder_params;

typedef struct nc_render_args {
  int32_t abi_version;   /* NC_ABI_VERSION */
  int32_t stage;         /* enum nc_stage */
  int64_t n_rays;
  int32_t n_strat;       /* N_samples (configs/nice_slam.yaml:122) */
  int32_t n_surf;        /* N_surface; must be 0 when gt_depth == NULL or stage == COARSE */
  int32_t flags;         /* NC_SAVE_FOR_BACKWARD (autograd: the graph requires grad) */
  int32_t lindisp;       /* ABI v9: 1 = stratified depths linear in disparity (Renderer.py:208-209) */
  const float* rays_o;   /* [N,3] */
  const float* rays_d;   /* [N,3] */
  const float* gt_depth; /* [N] or NULL */
  const float* depth_max;/* optional device scalar: batch-global max(gt_depth) (multi-GPU) */
  double bound[3][2];    /* renderer bound (Renderer.py:32): ray box and in-bound mask */
  float t_strat[NC_MAX_SAMPLES]; /* torch.linspace(0,1,n_strat) float32 */
  double t_surf[NC_MAX_SURF];    /* torch.linspace(0,1,n_surf).double() */
  nc_grid grids[4];              /* indexed by enum nc_decoder */
  nc_decoder_params dec[4];      /* indexed by enum nc_decoder */
  /* forward outputs */
  double* depth;  /* [N] */
  double* var;    /* [N] (uncertainty) */
  float* color;   /* [N,3] */
  /* backward inputs (NULL = zero upstream gradient) */
  const double* g_depth;
  const double* g_var;
  const float* g_color;
  /* backward outputs (NULL = not wanted) */
  float* g_rays_o; /* [N,3] */
  float* g_rays_d; /* [N,3] */
  /* fused rendering loss (loss != NC_LOSS_NONE): forward writes *loss_out (float64
   * device scalar, the reference's value incl. its float32 colour sum); backward adds
   * (*g_loss) * d loss / d (depth, colour) to g_depth / g_color (uncertainty enters the
   * tracker loss detached, as in the reference).  NC_LOSS_MAPPER with
   * NC_SAVE_FOR_BACKWARD (and not NC_DETERMINISTIC): the forward also forms the loss's
   * d raw for d loss = 1 and the backward scales it by *g_loss when that is the only
   * upstream gradient (no k_loss / k_composite_bwd); *loss_out is then the float64
   * per-workgroup partials added in block order by the last workgroup (fixed order,
   * identical run to run; w_color applied once to the float32 colour total). */
  int32_t loss;             /* NC_LOSS_* */
  int32_t loss_flags;       /* NC_LOSS_COLOR | NC_LOSS_DYNAMIC */
  double w_color;           /* w_color_loss (applied in float32, as the reference) */
  const float* loss_depth;  /* [N] target depth (batch_gt_depth; the coarse mapper renders
                               without gt_depth but its loss still uses it) */
  const float* loss_color;  /* [N,3] target colour; required with NC_LOSS_COLOR */
  double* loss_out;         /* device scalar */
  const double* g_loss;     /* device scalar upstream gradient of the loss (NULL = 0) */
  /* optional (ABI v4): the forward zero-fills grad_zero[0 .. grad_zero_floats) beside its
   * grid gathers -- e.g. the gradient buffer the backward will accumulate the grids'
   * gradients into -- instead of the caller launching a fill (16-B aligned, multiple
   * of 4 floats). */
  float* grad_zero;
  int64_t grad_zero_floats;
  /* hierarchical sampling, N_importance > 0 (ABI v6; src/utils/Renderer.py:239-259):
   * the first pass writes its sorted sample depths and compositing weights (z_out,
   * weights_out: [N][S]); sample_pdf (nc_sample_pdf) draws N_importance depths from
   * them; the second pass takes those as z_extra ([N][n_extra], no gradient) and
   * renders the sorted union of its own samples and them (S = n_strat + n_surf +
   * n_extra <= NC_MAX_SAMPLES). */
  const double* z_extra;
  int32_t n_extra;
  int32_t reserved3;
  double* z_out;
  float* weights_out;
  /* ABI v9: perturb > 0 (Renderer.py:211-219): the stratified depths are jittered inside
   * their intervals, z = lower + (upper - lower) * t_rand (float64 arithmetic), with the
   * caller's uniform draws t_rand [N][n_strat] float32 (the reference's
   * torch.rand(z_vals.shape)); NULL = no perturbation. */
  const float* t_rand;
  /* ABI v10: per-ray validity -- the callers' bbox pre-filter (src/Tracker.py:100-111,
   * src/Mapper.py:580-596) as a mask instead of a boolean-index compaction (a host sync).
   * A ray with ray_valid[i] == 0 is dropped: it is left out of the batch-global
   * max(gt_depth) (Renderer.py:157, :194), of the fused loss and of the Tracker's
   * handle_dynamic median; its depth / var / colour (and weights_out) are written as 0,
   * it adds nothing to any grid or decoder gradient and its ray gradients are 0.  The
   * kept rays' outputs, the loss and every gradient are those of rendering the compacted
   * batch (up to the summation order of the float reductions).  The samples of dropped
   * rays are still evaluated (fixed shapes: the call stays graph-capturable); non-finite
   * sample depths / points of dropped rays are replaced by 0.  NULL = every ray kept. */
  const uint8_t* ray_valid;
} nc_render_args;

typedef struct nc_points_args {
  int32_t abi_version;
  int32_t stage;
  int64_t n_points;
  int32_t flags;           /* NC_SAVE_FOR_BACKWARD */
  int32_t reserved;
  const double* pts;       /* [P,3] float64 (float32 callers convert) */
  nc_grid grids[4];
  nc_decoder_params dec[4];
  float* raw;              /* [P,4] output */
  const float* g_raw;      /* [P,4] upstream gradient (backward) */
  double* g_pts;           /* [P,3] or NULL */
} nc_points_args;

/* Training-ray sampling of one or more camera frames (ABI v4).  Replaces, in one
 * launch over all frames of an iteration:
 *   src/common.py:74-89   get_rays_from_uv (dirs = ((i-cx)/fx, -(j-cy)/fy, -1),
 *                         rays_d = sum(dirs * c2w[:3,:3], -1), rays_o = c2w[:3,3])
 *   src/common.py:92-108  select_uv (gather of the chosen pixels' depth / colour)
 *   src/common.py:111-137 get_sample_uv / get_samples (region H0..H1 x W0..W1; pixel
 *                         k of the region is (i, j) = (W0 + k % (W1-W0), H0 + k / (W1-W0)))
 *   src/Tracker.py:100-107, src/Mapper.py:580-591  the bbox pre-filter
 *                         inside = min_axis max_side (bound - o) / d >= gt_depth
 *                         (float64, NaN -> outside)
 * The caller draws the pixel indices (torch.randint, as select_uv does) and, when
 * the reference compacts the batch with `inside`, does that itself.  Backward:
 * d c2w[f] (rows 0..2: d R | d t) from d rays_o / d rays_d, summed over the frame's
 * rays in a fixed order. */
#define NC_POSE_F32 0
#define NC_POSE_F64 1
typedef struct nc_sample_args {
  int32_t abi_version;
  int32_t pose_dtype;        /* NC_POSE_F32 / NC_POSE_F64 (the c2w tensor's dtype) */
  int64_t n_frames;          /* F */
  int64_t n_per_frame;       /* n rays drawn per frame */
  int64_t H0, H1, W0, W1;    /* sampling region (get_samples' arguments) */
  float fx, fy, cx, cy;      /* intrinsics, as the float32 scalars torch applies them */
  const void* c2w;           /* [F] camera-to-world poses, rows 0..2 used */
  int64_t c2w_stride[3];     /* frame, row, column strides (elements) */
  const int64_t* indices;    /* [F][n] flat index into the region, row-major */
  const float* pix_i;        /* optional [F][n] float pixel columns / rows instead of indices */
  const float* pix_j;        /*   (get_rays_from_uv on caller uv; no depth / colour gather) */
  const int64_t* frame_ids;  /* optional [F]: image slot of pose f in depth / color (a resident
                                keyframe image stack); NULL = slot f */
  const float* depth;        /* [K] depth images [H][W], NULL = no depth output */
  int64_t depth_stride[3];   /* frame, row, column */
  const float* color;        /* [K] colour images [H][W][3], NULL = no colour output */
  int64_t color_stride[4];   /* frame, row, column, channel */
  const double* bound;       /* [3][2] scene bound for the pre-filter, or NULL */
  /* forward outputs ([F*n] rows, frame-major; rays in the pose dtype) */
  void* rays_o;              /* [F*n][3] */
  void* rays_d;              /* [F*n][3] */
  float* gt_depth;           /* [F*n] (needs depth) */
  float* gt_color;           /* [F*n][3] (needs color) */
  uint8_t* inside;           /* [F*n] bbox pre-filter mask (needs bound and depth) */
  /* backward */
  const void* g_rays_o;      /* [F*n][3] pose dtype, NULL = 0 */
  const void* g_rays_d;      /* [F*n][3] pose dtype, NULL = 0 */
  void* g_c2w;               /* [F][3][4] contiguous, pose dtype (written), or NULL with g_cam */
  /* ABI v11: the Tracker's camera tensor instead of c2w (src/common.py:163-176
   * get_camera_from_tensor: [qr, qi, qj, qk, tx, ty, tz] -> [quad2rotation(q) | t], with
   * two_s = 2 / |q|^2, common.py:137-160), so that a tracking iteration needs no torch ops
   * between the optimiser's camera tensor and the rays; the backward then writes d cam. */
  const void* cam;           /* [F][7] pose dtype, or NULL (then c2w) */
  int64_t cam_stride[2];     /* frame, element strides */
  void* g_cam;               /* [F][7] contiguous, pose dtype (written by the backward when cam) */
} nc_sample_args;

int nc_sample_rays_forward(const nc_sample_args* args, void* stream);
int nc_sample_rays_backward(const nc_sample_args* args, void* stream);

/* Frustum feature selection (ABI v4): Mapper.get_mask_from_c2w (src/Mapper.py:100-187)
 * for one grid on the device.  Per voxel (x, y, z) with world point (xs[x], ys[y],
 * zs[z]) -- the caller's torch.linspace tables, as the reference builds them --
 *   cam = w2c @ [p, 1] (float32), cam.x *= -1, uv = K @ cam (float64), z = uv.z + 1e-5,
 *   (u, v) = float32(uv.xy / z), d = cv2.remap(depth, u, v, INTER_LINEAR) (OpenCV 4.5:
 *   5-bit fixed-point sub-pixel weights, constant-0 border), d == 0 -> max over all d,
 *   mask = 0 < u < W & 0 < v < H & 0 <= -z <= d + 0.5  |  |p - c2w[:3,3]|^2 < 0.25.
 * Output in the grid's own [D][H][W] = [z][y][x] order (the reference returns the
 * [x][y][z] transpose, Mapper.py:185, and permutes it back at :394). */
typedef struct nc_frustum_args {
  int32_t abi_version;
  int32_t reserved;
  int64_t nx, ny, nz;          /* grid size along x, y, z (val_shape[2], [1], [0]) */
  const float* xs;             /* [nx] world x of the voxel columns (torch.linspace, float32) */
  const float* ys;             /* [ny] */
  const float* zs;             /* [nz] */
  float w2c[16];               /* np.linalg.inv(c2w) in float32, row-major 4x4 */
  float cam_o[3];              /* c2w[:3, 3] (float32) */
  float reserved2;
  double fx, fy, cx, cy;       /* intrinsics (float64, numpy's K) */
  const float* depth;          /* [H][W] float32 depth image */
  int64_t H, W;
  int64_t depth_stride[2];     /* row, column (elements) */
  uint8_t* mask;               /* [nz][ny][nx] output (bool) */
  uint32_t* scratch;           /* one uint32 of device scratch (max depth) */
} nc_frustum_args;

int nc_frustum_mask(const nc_frustum_args* args, void* stream);

/* Frustum feature selection's masked grid rows (ABI v8, additive): the Mapper keeps the
 * voxels inside the frame's frustum as one optimisable tensor and writes it into the grid
 * every iteration and back after the optimiser step (src/Mapper.py:393-404 val[mask]
 * .clone(), :491-500 val[mask] = val_grad, :633-642 the write-back; the backward of
 * that index_put is grad[mask]).  Here the mask is the list of its voxels, rows[n]
 * (ascending voxel index z*H*W + y*W + x, as mask.nonzero() gives them, computed once per
 * frame), and the optimisable tensor is laid out as ATen's val[mask] for the mask
 * repeated over the C channels: packed[c * n + i] = grid[0, c, voxel rows[i]].
 *   NC_ROWS_GATHER   packed <- grid rows   (val[mask], grad[mask])
 *   NC_ROWS_SCATTER  grid rows <- packed   (val[mask] = val_grad)
 *   NC_ROWS_ZERO     grid rows <- 0        (the index_put backward's gradient of val)
 * grid: [1, C, D, H, W] float32 with any strides (channels-last: one 128-B row per
 * voxel, transposed through LDS).  Plain copies: bit-identical to ATen's. */
#define NC_ROWS_GATHER 0
#define NC_ROWS_SCATTER 1
#define NC_ROWS_ZERO 2
typedef struct nc_grid_rows_args {
  int32_t abi_version;
  int32_t op;                  /* NC_ROWS_* */
  int64_t n_rows;
  const int64_t* rows;         /* [n_rows] voxel indices, each < D*H*W */
  float* grid;                 /* element (c, z, y, x) at c*stride[0] + z*stride[1] + y*stride[2] + x*stride[3] */
  int64_t channels;            /* C */
  int64_t dims[3];             /* D, H, W */
  int64_t stride[4];           /* elements */
  float* packed;               /* [C][n_rows] */
} nc_grid_rows_args;

int nc_grid_rows(const nc_grid_rows_args* args, void* stream);

/* Hierarchical (importance) sampling, sample_pdf (src/common.py:19-63), as
 * render_batch_ray applies it when N_importance > 0 (src/utils/Renderer.py:244-250):
 * per ray, N inverse-CDF samples of the piecewise-constant pdf weights + 1e-5 over
 * bins (float64 [n_rays][n_bins], the mid-points of the sorted sample depths;
 * weights float32 [n_rays][n_bins - 1]).  u = linspace(0, 1, N) when det, else the
 * caller's uniform draw (float32 [n_rays][N]).  n_bins, N <= NC_MAX_SAMPLES.
 * (ABI v5) */
typedef struct nc_pdf_args {
  int32_t abi_version;
  int32_t det;             /* 1: u = torch.linspace(0, 1, n_samples) */
  int64_t n_rays;
  int64_t n_bins;          /* >= 2 */
  int64_t n_samples;       /* N_importance */
  const double* bins;      /* [n_rays][n_bins], row stride bins_stride */
  int64_t bins_stride;
  const float* weights;    /* [n_rays][n_bins - 1], row stride weights_stride */
  int64_t weights_stride;
  const float* u;          /* [n_rays][n_samples] or NULL (det) */
  int64_t u_stride;
  double* samples;         /* [n_rays][n_samples] output */
  int64_t samples_stride;
} nc_pdf_args;

int nc_sample_pdf(const nc_pdf_args* args, void* stream);

/* Sparse gradient rows of one grid (ABI v5; see nc_grid). */
typedef struct nc_sparse_rows {
  int32_t* grad_rows;   /* [n_voxels] voxel -> row map */
  int64_t n_voxels;     /* D*H*W */
  int64_t* row_voxel;   /* [capacity] */
  int32_t* row_count;   /* device scalar */
  int64_t capacity;
  float* values;        /* [capacity][32] gradient rows */
} nc_sparse_rows;

/* Reset the map entries of the claimed rows to -1 and *row_count to 0 (the sparse
 * counterpart of zeroing grid.grad; the rows' values are zeroed when re-claimed). */
int nc_sparse_rows_clear(const nc_sparse_rows* rows, void* stream);

/* Multi-rank union of the touched-voxel sets before the gradient sum (RCCL):
 * all_voxel[r * rank_capacity + i] for i < all_count[r] are rank r's rows (the
 * all-gathered row_voxel / row_count of every rank, this one included).  Writes
 * `out`: the union, ascending by voxel -- identical on every rank -- as out->row_voxel
 * / *out->row_count, out->values = this rank's gradient rows permuted into that
 * order (zero where this rank has none), and the shared map in->grad_rows ==
 * out->grad_rows re-pointed to the new rows.  out->capacity >= the union's size
 * (world * rank_capacity always suffices).  Scratch: nc_sparse_merge_temp_bytes. */
size_t nc_sparse_merge_temp_bytes(int64_t n_keys, int64_t n_voxels);
int nc_sparse_rows_merge(const nc_sparse_rows* in, const nc_sparse_rows* out, const int64_t* all_voxel,
                         const int32_t* all_count, int32_t world, int64_t rank_capacity, void* temp,
                         size_t temp_bytes, void* stream);

/* Optimiser step of the Mapper (torch.optim.Adam over the grids and the colour decoder,
 * src/Mapper.py:462-485 param groups, :625 optimizer.step()).  (ABI v7)
 *   NC_ADAM_DENSE: param/grad/exp_avg/exp_avg_sq are n contiguous floats; the arithmetic of
 *     torch.optim.Adam(fused=True) (ATen fused_adam_utils.cuh adam_math: ORIGINAL mode,
 *     weight_decay added to the gradient, no amsgrad / maximize).  step = the step count
 *     after its increment (1 at the first step).
 *   NC_ADAM_SPARSE_ROWS: torch.optim.SparseAdam's rule (torch/optim/_functional.py
 *     sparse_adam) on the rows of a sparse grid gradient (nc_sparse_rows): grad = the
 *     [row_capacity][32] values, row_voxel / *row_count the touched voxels; param and
 *     moments addressed as voxel * voxel_stride + channel * channel_stride.  Untouched
 *     voxels are left as they are (lazy).  weight_decay must be 0, as SparseAdam has none. */
#define NC_ADAM_DENSE 0
#define NC_ADAM_SPARSE_ROWS 1
typedef struct nc_adam_args {
  int32_t abi_version;
  int32_t mode;               /* NC_ADAM_* */
  int64_t n;                  /* dense: number of elements */
  float* param;
  const float* grad;          /* dense: [n]; rows: [row_capacity][32] */
  float* exp_avg;
  float* exp_avg_sq;
  const int64_t* row_voxel;   /* rows: [row_capacity] */
  const int32_t* row_count;   /* rows: device scalar */
  int64_t row_capacity;
  int64_t voxel_stride;       /* rows: channels-last 32, NCDHW 1 */
  int64_t channel_stride;     /* rows: channels-last 1, NCDHW D*H*W */
  double lr, beta1, beta2, eps, weight_decay;
  double step;
} nc_adam_args;

int nc_adam_step(const nc_adam_args* args, void* stream);

/* The dense rule over many parameters in one launch per NC_ADAM_MAX_SEGMENTS
 * (torch.optim.Adam(fused=True) steps all parameters of the optimiser together):
 * segment i is (param, grad, exp_avg, exp_avg_sq, n) with its group's lr /
 * weight_decay and its own step count; betas and eps come from `args` (mode and
 * the pointer fields of `args` are ignored).  (ABI v7) */
#define NC_ADAM_MAX_SEGMENTS 32
typedef struct nc_adam_segment {
  float* param;
  const float* grad;
  float* exp_avg;
  float* exp_avg_sq;
  int64_t n;
  double lr, weight_decay, step;
  float* step_dev;      /* optional: the step count in device memory (float32, as torch's
                           capturable state): incremented by the call, then used instead of
                           `step` -- a graph-captured step sees the live count */
} nc_adam_segment;

int nc_adam_step_multi(const nc_adam_args* args, const nc_adam_segment* segments, int32_t n_segments,
                       void* stream);

int nc_abi_version(void);
const char* nc_last_error(void);

/* The sources this binary was compiled from: the first 16 hex digits of a sha256 over
 * csrc/ and this header (nicecore/build.py:source_hash, passed as -DNC_SRC_HASH).  The
 * Python binding refuses a library whose id differs from the tree it is loaded from. */
const char* nc_build_id(void);

/* Number of floats in a decoder's flat parameter vector (58,956 over all four). */
int64_t nc_param_count(int decoder);

/* sizeof() of the ABI structs, for binding-layout checks:
 * 0 nc_render_args, 1 nc_points_args, 2 nc_grid, 3 nc_decoder_params, 4 nc_sample_args, 5 nc_frustum_args,
 * 6 nc_sparse_rows, 7 nc_pdf_args, 8 nc_adam_args, 9 nc_adam_segment, 10 nc_imap_render_args,
 * 11 nc_imap_points_args, 12 nc_imap_params, 13 nc_grid_rows_args. */
size_t nc_struct_size(int which);

size_t nc_render_workspace_bytes(const nc_render_args* args);
int nc_render_forward(const nc_render_args* args, void* workspace, size_t workspace_bytes,
                      void* stream);
int nc_render_backward(const nc_render_args* args, void* workspace, size_t workspace_bytes,
                       void* stream);
/* The decoder weight gradients a backward with NC_DEFER_PARAM_GRADS left out: same args
 * (the decoders' grad pointers), same workspace, before the next forward on it. (ABI v7) */
int nc_render_backward_params(const nc_render_args* args, void* workspace, size_t workspace_bytes,
                              void* stream);

/* Kernel timing with HIP events recorded on the launch stream around every
 * launch of the kernels in `kernel_mask` (bit i = kernel id i, see
 * nc_kernel_name).  nc_timing_stop synchronises the recorded events and returns
 * per-kernel total milliseconds and launch counts (arrays of max_kernels). */
int nc_timing_start(uint32_t kernel_mask);
int nc_timing_stop(double* total_ms, int64_t* launches, int max_kernels);
const char* nc_kernel_name(int kernel_id);

/* NICE_CORE_PROFILE=1 in the environment: every kernel launch of the process is event-timed
 * on its stream (launches enqueued during a graph capture excepted) and folded into
 * per-kernel totals; nc_profile_report prints launches / total / average per kernel to
 * stderr (the Python binding calls it at interpreter exit).  Returns 0 (also when the
 * flag is off), negative if an event could not be read. */
int nc_profile_report(void);

size_t nc_points_workspace_bytes(const nc_points_args* args);
int nc_points_forward(const nc_points_args* args, void* workspace, size_t workspace_bytes,
                      void* stream);
int nc_points_backward(const nc_points_args* args, void* workspace, size_t workspace_bytes,
                       void* stream);

/* ---- iMAP* (ABI v8) ------------------------------------------
 * The single-MLP scene model of configs/imap.yaml: get_model(nice=False) builds
 * MLP(dim=3, c_dim=0, color=True, hidden_size=256, skips=[], n_blocks=4)
 * (src/conv_onet/config.py:28-32, decoder.py:116-219): emb = sin(p.float() @ B)
 * (B [3,93]), h_0 = relu(W_0 emb + b_0) (W_0 [256,93]), h_l = relu(W_l h_{l-1} + b_l)
 * (l = 1..3, [256,256]), raw = W_out h_3 + b_out (W_out [4,256]).  Rendering uses
 * volume density (occupancy: False): alpha = 1 - exp(-relu(raw[...,3]) * dists),
 * dists = (z_{i+1} - z_i).float() (1e10 after the last sample) * ||rays_d||
 * (src/common.py:232-247); points outside the renderer bound get raw[...,3] = 100
 * (Renderer.py:87).  Replaces Renderer.render_batch_ray (Renderer.py:95-262) with
 * nice=False and Renderer.eval_points (:36-93, decoders(pi, c_grid=None)). */
#define NC_IMAP_HIDDEN 256
typedef struct nc_imap_params {
  const float* fourier_B; /* [3, 93] embedder._B */
  const float* lin_w[4];  /* pts_linears[l].weight: [256, 93], [256, 256] x 3 */
  const float* lin_b[4];  /* [256] */
  const float* out_w;     /* output_linear.weight [4, 256] */
  const float* out_b;     /* [4] */
  float* grad;            /* flat gradient in nn.Module.parameters() order (222,747 floats), or NULL */
} nc_imap_params;

typedef struct nc_imap_render_args {
  int32_t abi_version;   /* NC_ABI_VERSION */
  int32_t flags;         /* NC_SAVE_FOR_BACKWARD */
  int64_t n_rays;
  int32_t n_strat;       /* N_samples (configs/imap.yaml:107); N_surface is 0 for iMAP* */
  int32_t n_extra;       /* importance depths merged into the samples (second pass) */
  const float* rays_o;   /* [N,3] */
  const float* rays_d;   /* [N,3] */
  const float* gt_depth; /* [N] or NULL */
  const float* depth_max;/* optional device scalar: batch-global max(gt_depth) */
  double bound[3][2];
  float t_strat[NC_MAX_SAMPLES];
  nc_imap_params dec;
  double* depth;         /* [N] */
  double* var;           /* [N] */
  float* color;          /* [N,3] */
  const double* g_depth; /* backward inputs (NULL = zero) */
  const double* g_var;
  const float* g_color;
  float* g_rays_o;       /* backward outputs (NULL = not wanted) */
  float* g_rays_d;
  const double* z_extra; /* [N][n_extra] (ABI v6 semantics) */
  double* z_out;         /* optional [N][S] */
  float* weights_out;    /* optional [N][S] */
} nc_imap_render_args;

typedef struct nc_imap_points_args {
  int32_t abi_version;
  int32_t flags;         /* NC_SAVE_FOR_BACKWARD */
  int64_t n_points;
  const double* pts;     /* [P,3] float64 */
  nc_imap_params dec;
  float* raw;            /* [P,4] decoder output (no bound mask: Renderer.eval_points applies it) */
  const float* g_raw;    /* [P,4] upstream gradient (backward) */
  double* g_pts;         /* [P,3] or NULL */
} nc_imap_points_args;

int64_t nc_imap_param_count(void);
size_t nc_imap_render_workspace_bytes(const nc_imap_render_args* args);
int nc_imap_render_forward(const nc_imap_render_args* args, void* workspace, size_t workspace_bytes, void* stream);
int nc_imap_render_backward(const nc_imap_render_args* args, void* workspace, size_t workspace_bytes, void* stream);
size_t nc_imap_points_workspace_bytes(const nc_imap_points_args* args);
int nc_imap_points_forward(const nc_imap_points_args* args, void* workspace, size_t workspace_bytes, void* stream);
int nc_imap_points_backward(const nc_imap_points_args* args, void* workspace, size_t workspace_bytes, void* stream);
/* Byte offset inside the workspace of the saved hidden activations h_layer = relu(z)
 * (layer 0..3, [n_points][256] float32, point-major) that nc_imap_points_forward wrote:
 * read-only introspection (the tests score weight gradients against a float64 truth
 * evaluated on the same ReLU branches).  Returns -1 for a bad layer or arguments. */
int64_t nc_imap_points_activation_offset(const nc_imap_points_args* args, int layer);

#ifdef __cplusplus
}
#endif
#endif /* NICECORE_H */
