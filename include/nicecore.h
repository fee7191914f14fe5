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

#define NC_ABI_VERSION 3
#define NC_MAX_SAMPLES 64 /* n_strat + n_surf per ray (one wavefront per ray) */
#define NC_MAX_SURF 32

/* nc_*_args.flags */
#define NC_SAVE_FOR_BACKWARD 1
/* Grid gradients by an ordered reduction instead of float atomics: bit-identical run
 * to run, summed per voxel in the reference's order (ascending point, corner).  Set it
 * on the forward (it sizes the workspace) and keep it for the backward. */
#define NC_DETERMINISTIC 2

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
 * (torch.channels_last_3d) is the fast path. */
typedef struct nc_grid {
  const float* data;
  float* grad;            /* NULL: no gradient wanted for this grid */
  int64_t dims[3];        /* D, H, W */
  int64_t stride[4];      /* C, D, H, W strides of data */
  int64_t grad_stride[4]; /* C, D, H, W strides of grad */
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
  int32_t reserved;      /* 0 */
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
   * tracker loss detached, as in the reference). */
  int32_t loss;             /* NC_LOSS_* */
  int32_t loss_flags;       /* NC_LOSS_COLOR | NC_LOSS_DYNAMIC */
  double w_color;           /* w_color_loss (applied in float32, as the reference) */
  const float* loss_depth;  /* [N] target depth (batch_gt_depth; the coarse mapper renders
                               without gt_depth but its loss still uses it) */
  const float* loss_color;  /* [N,3] target colour; required with NC_LOSS_COLOR */
  double* loss_out;         /* device scalar */
  const double* g_loss;     /* device scalar upstream gradient of the loss (NULL = 0) */
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

int nc_abi_version(void);
const char* nc_last_error(void);

/* Number of floats in a decoder's flat parameter vector (58,956 over all four). */
int64_t nc_param_count(int decoder);

/* sizeof() of the ABI structs, for binding-layout checks:
 * 0 nc_render_args, 1 nc_points_args, 2 nc_grid, 3 nc_decoder_params. */
size_t nc_struct_size(int which);

size_t nc_render_workspace_bytes(const nc_render_args* args);
int nc_render_forward(const nc_render_args* args, void* workspace, size_t workspace_bytes,
                      void* stream);
int nc_render_backward(const nc_render_args* args, void* workspace, size_t workspace_bytes,
                       void* stream);

/* Kernel timing with HIP events recorded on the launch stream around every
 * launch of the kernels in `kernel_mask` (bit i = kernel id i, see
 * nc_kernel_name).  nc_timing_stop synchronises the recorded events and returns
 * per-kernel total milliseconds and launch counts (arrays of max_kernels). */
int nc_timing_start(uint32_t kernel_mask);
int nc_timing_stop(double* total_ms, int64_t* launches, int max_kernels);
const char* nc_kernel_name(int kernel_id);

size_t nc_points_workspace_bytes(const nc_points_args* args);
int nc_points_forward(const nc_points_args* args, void* workspace, size_t workspace_bytes,
                      void* stream);
int nc_points_backward(const nc_points_args* args, void* workspace, size_t workspace_bytes,
                       void* stream);

#ifdef __cplusplus
}
#endif
#endif /* NICECORE_H */
