// nc_abi.hip — extern "C" entry points of libnicecore.so (see include/nicecore.h).
//
// Plans the launches of one render_batch_ray forward / backward:
//   forward : [k_depth_max] -> k_ray_setup -> k_grid_gather -> k_mlp_fwd (all
//             decoders of the stage in one launch) -> k_composite_fwd -> [k_loss]
//   backward: k_composite_bwd -> k_mlp_dx (incl. the trilinear backward) ->
//             [k_mlp_dw -> k_param_reduce] -> [k_ray_grads]
// Everything is enqueued on the caller's stream; no host synchronisation, no
// device allocation (graph-capturable).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "nc_device.h"
#include "nc_internal.h"
#include "nc_wimage.h"

using namespace nc;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

int check_hip(int e, const char* what) {
  if (e != (int)hipSuccess) return fail(-4, std::string(what) + ": " + hipGetErrorString((hipError_t)e));
  return 0;
}

// ---- optional per-kernel event timing (nc_timing_start / nc_timing_stop) ----
enum KernelId {
  KID_DEPTH_MAX = 0, KID_RAY_SETUP, KID_MLP_FWD, KID_COMPOSITE_FWD, KID_COMPOSITE_BWD, KID_MLP_DX,
  KID_PARAM_REDUCE, KID_RAY_GRADS, KID_POINTS_ASSEMBLE, KID_POINTS_SPLIT, KID_POINTS_GRADS, KID_GRID_BWD, KID_MLP_DW,
  KID_GRID_GATHER, KID_LOSS, KID_DET_SCATTER, KID_SAMPLE_RAYS, KID_SAMPLE_POSE_GRAD, KID_FRUSTUM, KID_ROWS_CLEAR,
  KID_ROWS_MERGE, KID_ROWS_CLAIM, KID_PARAM_RAY, KID_SAMPLE_PDF, KID_ADAM, KID_IMAP_GEMM, KID_IMAP_FOURIER, KID_GRID_ROWS,
  KID_COMPOSITE_FWD_LOSS, KID_COUNT
};
const char* kKernelNames[KID_COUNT] = {"k_depth_max", "k_ray_setup", "k_mlp_fwd", "k_composite_fwd",
                                       "k_composite_bwd", "k_mlp_dx", "k_param_reduce", "k_ray_grads",
                                       "k_points_assemble", "k_points_split_grad", "k_points_grads", "k_grid_bwd",
                                       "k_mlp_dw", "k_grid_gather", "k_loss", "k_det_scatter",
                                       "k_sample_rays", "k_sample_pose_grad", "k_frustum_mask", "k_rows_clear", "k_rows_merge", "k_rows_compact", "k_param_ray_reduce", "k_sample_pdf", "k_adam",
                                       "k_imap_gemm", "k_imap_fourier", "k_grid_rows", "k_composite_fwd_loss"};
struct TimedLaunch {
  hipEvent_t b, e;
  int id;
};
struct Timing {
  uint32_t mask = 0;
  std::vector<TimedLaunch> used;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> pool;
} g_timing;

// NICE_CORE_PROFILE=1: every timed launch of the process is event-timed on
// its stream and folded into per-kernel totals; nc_profile_report() prints them (the Python
// binding calls it at exit).  Launches enqueued while the stream is being captured into a
// graph are not timed (counted apart).  Every 2,048 pending launches the older half is
// synchronised and folded, so a long run keeps a bounded event list.
struct Profile {
  int on = -1;
  std::vector<TimedLaunch> pending;
  double total_ms[KID_COUNT] = {};
  int64_t launches[KID_COUNT] = {};
  int64_t captured = 0;
} g_prof;

bool profile_on() {
  if (g_prof.on < 0) {
    const char* e = std::getenv("NICE_CORE_PROFILE");
    g_prof.on = (e && e[0] == '1' && e[1] == 0) ? 1 : 0;
  }
  return g_prof.on == 1;
}

bool take_events(std::pair<hipEvent_t, hipEvent_t>& ev) {
  if (!g_timing.pool.empty()) {
    ev = g_timing.pool.back();
    g_timing.pool.pop_back();
    return true;
  }
  return hipEventCreate(&ev.first) == hipSuccess && hipEventCreate(&ev.second) == hipSuccess;
}

int prof_fold(size_t n) {  // synchronise and fold the oldest n pending launches
  if (n > g_prof.pending.size()) n = g_prof.pending.size();
  int rc = 0;
  for (size_t k = 0; k < n; ++k) {
    const TimedLaunch& t = g_prof.pending[k];
    float ms = 0.f;
    if (hipEventSynchronize(t.e) != hipSuccess || hipEventElapsedTime(&ms, t.b, t.e) != hipSuccess) rc = -4;
    g_prof.total_ms[t.id] += ms;
    g_prof.launches[t.id] += 1;
    g_timing.pool.push_back({t.b, t.e});
  }
  g_prof.pending.erase(g_prof.pending.begin(), g_prof.pending.begin() + (long)n);
  return rc;
}

template <typename F>
int timed(int id, hipStream_t s, F&& launch) {
  const bool t = (g_timing.mask & (1u << id)) != 0;
  const bool p = profile_on();
  if (!t && !p) return launch();
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cap) == hipSuccess && cap != hipStreamCaptureStatusNone) {
    if (p) g_prof.captured++;  // events inside a graph capture: not timed
    return launch();
  }
  std::pair<hipEvent_t, hipEvent_t> et, ep;
  const bool ot = t && take_events(et), op = p && take_events(ep);
  if (ot) (void)hipEventRecord(et.first, s);
  if (op) (void)hipEventRecord(ep.first, s);
  const int rc = launch();
  if (op) (void)hipEventRecord(ep.second, s);
  if (ot) (void)hipEventRecord(et.second, s);
  if (ot) g_timing.used.push_back({et.first, et.second, id});
  if (op) {
    g_prof.pending.push_back({ep.first, ep.second, id});
    if (g_prof.pending.size() >= 2048) (void)prof_fold(1024);
  }
  return rc;
}

int cu_count() {
  static int cache[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cache[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cache[dev] = n;
  }
  return cache[dev];
}

size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

// up to this many rays every k_ray_setup workgroup reduces max(gt_depth) itself
// (<= 16 KB of L2 reads per workgroup) instead of a separate k_depth_max launch
constexpr int64_t kDmaxLocalRays = 4096;

struct Plan {
  int n_jobs = 0;
  Job jobs[MAX_JOBS];
  int occ_a = -1, occ_b = -1;
  bool has_rgb = false;
};

// decoder.py:341-370: which decoders a stage evaluates
int plan_stage(int stage, Plan& pl) {
  pl = Plan();
  auto add = [&](int kind) {
    Job& j = pl.jobs[pl.n_jobs];
    std::memset(&j, 0, sizeof(j));
    j.kind = kind;
    j.slot = pl.n_jobs;
    pl.n_jobs++;
  };
  switch (stage) {
    case NC_STAGE_COARSE: add(K_COARSE); pl.occ_a = 0; break;
    case NC_STAGE_MIDDLE: add(K_MID); pl.occ_a = 0; break;
    case NC_STAGE_FINE: add(K_FINE); add(K_MID); pl.occ_a = 0; pl.occ_b = 1; break;
    case NC_STAGE_COLOR: add(K_FINE); add(K_MID); add(K_COLOR); pl.occ_a = 0; pl.occ_b = 1; pl.has_rgb = true; break;
    default: return fail(-1, "nicecore: unknown stage " + std::to_string(stage));
  }
  return 0;
}

int check_grid(const nc_grid& g, const char* name) {
  if (!g.data) return fail(-1, std::string("nicecore: grid ") + name + " is required by this stage but NULL");
  for (int k = 0; k < 3; ++k)
    if (g.dims[k] < 1) return fail(-1, std::string("nicecore: grid ") + name + " has an empty dimension");
  // the kernels index voxels in int32 and take element strides as int32 (nc_device.h Corners)
  for (int k = 0; k < 3; ++k)
    if (g.dims[k] > (INT32_MAX >> 1)) return fail(-1, std::string("nicecore: grid ") + name + " dimension >= 2^30");
  for (int k = 0; k < 4; ++k) {
    if (g.stride[k] < 0 || g.stride[k] > INT32_MAX)
      return fail(-1, std::string("nicecore: grid ") + name + " has an element stride outside [0, 2^31)");
    if (g.grad && !g.grad_rows && (g.grad_stride[k] < 0 || g.grad_stride[k] > INT32_MAX))
      return fail(-1, std::string("nicecore: grid ") + name + " gradient has an element stride outside [0, 2^31)");
  }
  if (g.grad_rows) {  // sparse gradient rows (ABI v5)
    if (!g.row_voxel || !g.row_count || g.row_capacity < 1 || !g.grad ||
        (reinterpret_cast<uintptr_t>(g.grad) & 15))
      return fail(-1, std::string("nicecore: grid ") + name +
                          " has grad_rows but no 16-B aligned gradient rows, row_voxel, row_count or capacity");
    if (g.row_capacity > INT32_MAX || g.dims[0] * g.dims[1] * g.dims[2] > INT32_MAX)
      return fail(-1, std::string("nicecore: grid ") + name + ": sparse rows need < 2^31 voxels and rows");
  }
  return 0;
}

int check_dec(const nc_decoder_params& d, int kind) {
  const bool xyz = kind != K_COARSE;
  for (int i = 0; i < 5; ++i)
    if (!d.lin_w[i] || !d.lin_b[i] || (xyz && (!d.fc_w[i] || !d.fc_b[i])))
      return fail(-1, "nicecore: decoder " + std::to_string(kind) + " has a NULL parameter pointer");
  if (!d.out_w || !d.out_b || (xyz && !d.fourier_B))
    return fail(-1, "nicecore: decoder " + std::to_string(kind) + " has a NULL parameter pointer");
  return 0;
}

const char* grid_name(int k) {
  static const char* n[4] = {"grid_coarse", "grid_middle", "grid_fine", "grid_color"};
  return n[k];
}

int check_models(const Plan& pl, const nc_grid* grids, const nc_decoder_params* dec) {
  for (int j = 0; j < pl.n_jobs; ++j) {
    const int k = pl.jobs[j].kind;
    if (int e = check_grid(grids[k], grid_name(k))) return e;
    if (k == K_FINE)
      if (int e = check_grid(grids[K_MID], grid_name(K_MID))) return e;
    if (int e = check_dec(dec[k], k)) return e;
  }
  return 0;
}

struct Ws {
  size_t dmax = 0, rflag = 0, wimg = 0, dximg = 0, z = 0, pts = 0, xyz = 0, pf = 0, occ = 0, rgb = 0, gocc = 0, grgb = 0, dpts = 0, slab = 0, rec = 0, feat = 0,
         gocc_b = 0, grgb_b = 0,  // fused mapper loss: d raw of a backward that is not d loss alone
         lpart = 0, lcount = 0,   // fused mapper loss: per-workgroup partial sums + done counter
         coef_d = 0, coef_c = 0, bslab = 0, dfeat = 0, dkey[2] = {0, 0}, dval[2] = {0, 0}, dw = 0, dpart = 0, dtemp = 0,
         dtemp_bytes = 0,
         total = 0;
  bool det = false;
  size_t jac = 0;
  bool has_jac = false;
  size_t claim_cnt = 0, claim_tmp = 0;  // sparse-row claims (nc_grid.grad_rows)
  int64_t claim_cap = 0;
  bool claims = false;
  int vbits = 0;
  int64_t dppad = 0;   // NC_DETERMINISTIC points per job in the entry arrays (det_ppad)
  int dsort_bits = 8;  // NC_DETERMINISTIC radix digit width (det_sort_bits)
  int64_t rec_off[MAX_JOBS] = {0, 0, 0};
  bool save = false;
  bool fuse = false;  // k_mlp_fwd gathers the grid features itself (no k_grid_gather, no feature buffer)
  int slab_wgs = 1;        // total k_mlp_dw workgroups (= slab rows)
  int32_t dw_off[MAX_JOBS + 1] = {0, 0, 0, 0};
  int64_t slab_stride = 0;
  int32_t bslab_rows = 0;  // k_mlp_dx workgroups per job (its grid x)
};

int fwd_grid_x(int64_t P, int n_jobs, int which);

// Split `total` resident workgroups over the jobs in proportion to their per-point
// cost (decoder MACs), each job at least 1 and at most its `blocks` work items;
// off[j]..off[j+1] are job j's workgroups of a 1-D grid, off[k > n_jobs] = off[n_jobs].
void split_wgs(int total, int64_t blocks, const Job* jobs, int n_jobs, int32_t* off, int (*cost)(int) = decoder_macs) {
  if (total < n_jobs) total = n_jobs;
  int64_t wsum = 0;
  for (int j = 0; j < n_jobs; ++j) wsum += cost(jobs[j].kind);
  off[0] = 0;
  int64_t acc = 0;
  for (int j = 0; j < n_jobs; ++j) {
    acc += cost(jobs[j].kind);
    int64_t n = (total * acc + wsum / 2) / wsum - off[j];  // rounded cumulative share
    if (n < 1) n = 1;
    if (n > blocks) n = blocks > 0 ? blocks : 1;
    off[j + 1] = off[j] + (int32_t)n;
  }
  for (int j = n_jobs + 1; j <= MAX_JOBS; ++j) off[j] = off[n_jobs];
}

// a grid whose corner rows k_mlp_fwd's fused gather reads as float4s (device grid_vec_ok)
static bool host_vec_ok(const nc_grid& G) {
  return G.data && G.stride[0] == 1 && (reinterpret_cast<uintptr_t>(G.data) & 15u) == 0 &&
         G.stride[1] % 4 == 0 && G.stride[2] % 4 == 0 && G.stride[3] % 4 == 0;
}

// every grid the stage's decoders look up (the fine decoder: also grid_middle) is
// channels-last: the forward's trilinear lookups can run inside k_mlp_fwd
static bool stage_fuse(const Plan& pl, const nc_grid* grids) {
  for (int j = 0; j < pl.n_jobs; ++j) {
    const int k = pl.jobs[j].kind;
    if (!host_vec_ok(grids[k]) || (k == K_FINE && !host_vec_ok(grids[K_MID]))) return false;
  }
  return true;
}

void layout(int64_t N, int64_t P, const Plan& pl, bool rays, bool save, bool loss, Ws& w, int vbits = -1,
            bool jac = false, bool claims = false, bool fuse = false, bool fused_loss = false) {
  size_t off = 0;
  auto take = [&](size_t bytes) {
    const size_t o = off;
    off = align256(off + bytes);
    return o;
  };
  w.dmax = take(16);
  w.rflag = take(4 * MAX_JOBS);  // MlpCtx::range_flag
  w.wimg = take((size_t)pl.n_jobs * WIMG_STRIDE);  // MlpCtx::wimg (nc_wimage.h)
  w.z = rays ? take((size_t)P * 8) : 0;
  w.pts = rays ? take((size_t)P * 24) : 0;
  w.xyz = take((size_t)pl.n_jobs * P * 16);
  w.pf = take((size_t)P * 16);
  w.occ = take((size_t)pl.n_jobs * P * 4);
  w.rgb = take((size_t)P * 12);
  w.gocc = take((size_t)P * 4);
  w.grgb = take((size_t)P * 12);
  w.dpts = take((size_t)pl.n_jobs * P * 24);
  w.jac = (save && jac) ? take((size_t)pl.n_jobs * P * 96 * 4) : 0;
  w.has_jac = save && jac;
  w.claims = save && claims;
  if (w.claims) {  // per-shard claim lists of k_grid_gather: every lane of a shard's waves fits
    const int64_t waves = (P * 16 + 255) / 256 * 4;  // gather waves of the widest job
    w.claim_cap = ((waves + CLAIM_SHARDS - 1) / CLAIM_SHARDS + 1) * 64;
    w.claim_cnt = take((size_t)MAX_JOBS * CLAIM_SHARDS * 4);
    w.claim_tmp = take((size_t)MAX_JOBS * CLAIM_SHARDS * w.claim_cap * 8);
  }
  if (loss) {  // per-ray loss derivatives, forward -> backward
    w.coef_d = take((size_t)N * 8);
    w.coef_c = take((size_t)N * 12);
  }
  if (fused_loss) {  // k_composite_fwd_loss's d raw (d loss = 1) stays in gocc / grgb for every
                     // loss-only backward of a retained graph; any other backward writes here
    w.gocc_b = take((size_t)P * 4);
    w.grgb_b = take((size_t)P * 12);
    w.lpart = take((size_t)fused_loss_blocks(N) * 16);
    w.lcount = take(16);
  }
  w.save = save;
  w.dximg = save ? take((size_t)pl.n_jobs * DXIMG_STRIDE) : 0;  // MlpCtx::dximg (k_mlp_dx's weights)
  // the fused gather (k_mlp_fwd) cannot claim sparse rows or save the Jacobian
  w.fuse = fuse && !w.claims && !w.has_jac;
  if (save) {
    int64_t r = 0;
    for (int j = 0; j < pl.n_jobs; ++j) {
      w.rec_off[j] = r;
      r += P * rec_stride(pl.jobs[j].kind);
    }
    w.rec = take((size_t)r * 4);
  } else if (!w.fuse) {  // forward only: k_grid_gather's features go to their own buffer
    int64_t f = 0;
    for (int j = 0; j < pl.n_jobs; ++j) {
      w.rec_off[j] = f;
      f += P * (pl.jobs[j].kind == K_FINE ? 64 : 32);
    }
    w.feat = take((size_t)f * 4);
  }
  const int64_t blocks = (P + 31) / 32;  // k_mlp_dw sub-chunks
  // one wave of resident workgroups over all jobs (floor: a 257th workgroup on a
  // 256-CU chip would run as a second, serial round), split by the decoders' cost
  split_wgs(cu_count() * mlp_blocks_per_cu(2), blocks, pl.jobs, pl.n_jobs, w.dw_off);
  w.slab_wgs = w.dw_off[pl.n_jobs];
  w.slab_stride = (max_param_count() + 63) & ~int64_t(63);
  w.slab = take((size_t)w.slab_wgs * w.slab_stride * 4);
  if (save) {  // k_mlp_dx's Fourier-B weight-gradient rows (MlpCtx::bslab)
    w.bslab_rows = fwd_grid_x(P, pl.n_jobs, 1);
    w.bslab = take((size_t)pl.n_jobs * w.bslab_rows * DX_BSLAB * 4);
  }
  if (save && vbits > 0) {  // NC_DETERMINISTIC grid-gradient buffers (nc_det.hip)
    const int64_t ne = (int64_t)pl.n_jobs * det_ppad(P) * 8;  // each job's points padded to a radix tile
    w.det = true;
    w.vbits = vbits;
    w.dppad = det_ppad(P);
    w.dfeat = take((size_t)pl.n_jobs * P * 32 * 4);
    for (int b = 0; b < 2; ++b) {
      w.dkey[b] = take((size_t)ne * 8);
      w.dval[b] = take((size_t)ne * 4);
    }
    w.dw = take((size_t)ne * 4);
    w.dpart = take((size_t)(ne + 8 * DET_DSUB - 1) / (8 * DET_DSUB) * 2 * 32 * 4);
    w.dsort_bits = det_sort_bits(vbits + 2);
    w.dtemp_bytes = det_sort_temp_bytes(ne, w.dsort_bits);
    w.dtemp = take(w.dtemp_bytes);
  }
  w.total = off;
}

template <typename T>
T* at(void* ws, size_t off) {
  return reinterpret_cast<T*>(reinterpret_cast<char*>(ws) + off);
}

void fill_mlp(MlpCtx& m, int64_t P, const Plan& pl, const nc_grid* grids, const nc_decoder_params* dec,
              const double* pts, void* ws, const Ws& w, bool need_coord) {
  std::memset(&m, 0, sizeof(m));
  m.P = P;
  m.n_jobs = pl.n_jobs;
  m.slab_wgs = w.slab_wgs;
  m.slab_stride = w.slab_stride;
  std::memcpy(m.dw_off, w.dw_off, sizeof(m.dw_off));
  {  // k_mlp_fwd split: one wave of resident workgroups, 16-point tiles per wave
    const int64_t per = fwd_threads(w.fuse) / 64 * 16 * FWD_TILES;
    split_wgs(cu_count() * mlp_blocks_per_cu(w.fuse ? 3 : 0), (P + per - 1) / per, pl.jobs, pl.n_jobs, m.fwd_off,
              fwd_tile_cost);
  }
  m.save_rec = w.save;
  for (int j = 0; j < pl.n_jobs; ++j) {
    m.jobs[j] = pl.jobs[j];
    const int k = pl.jobs[j].kind;
    m.jobs[j].rec_off = w.rec_off[j];
    if (w.save) {
      m.jobs[j].c_off = w.rec_off[j] + rec_feat_offset(k);
      m.jobs[j].c_stride = rec_stride(k);
    } else {
      m.jobs[j].c_off = w.rec_off[j];
      m.jobs[j].c_stride = k == K_FINE ? 64 : 32;
    }
    m.jobs[j].need_dw = dec[k].grad != nullptr;
    m.jobs[j].need_grid = grids[k].grad != nullptr;
    m.jobs[j].need_coord = need_coord;
    m.jobs[j].keep_h = 1;
  }
  {  // k_mlp_dw: the layout's workgroups go to the decoders that want a weight gradient
     // only (e.g. the Mapper's fix_fine: the color decoder alone); others get none
    Job sel[MAX_JOBS];
    int pos[MAX_JOBS], n = 0;
    for (int j = 0; j < pl.n_jobs; ++j)
      if (m.jobs[j].need_dw) {
        sel[n] = m.jobs[j];
        pos[n++] = j;
      }
    if (n > 0 && n < pl.n_jobs) {
      int32_t o[MAX_JOBS + 1];
      split_wgs(w.slab_wgs, (P + 31) / 32, sel, n, o);
      m.dw_off[0] = 0;
      for (int j = 0, q = 0; j < MAX_JOBS; ++j) {
        const bool own = q < n && pos[q] == j;
        m.dw_off[j + 1] = m.dw_off[j] + (own ? o[q + 1] - o[q] : 0);
        q += own ? 1 : 0;
      }
    }
  }
  std::memcpy(m.grids, grids, sizeof(m.grids));
  std::memcpy(m.dec, dec, sizeof(m.dec));
  m.share_mid = pl.n_jobs >= 2 && pl.jobs[0].kind == K_FINE && pl.jobs[1].kind == K_MID &&
                std::memcmp(dec[K_FINE].bound, dec[K_MID].bound, sizeof(dec[K_FINE].bound)) == 0;
  m.pts = pts;
  m.xyz = at<float4>(ws, w.xyz);
  m.pf = at<float4>(ws, w.pf);
  m.occ = at<float>(ws, w.occ);
  m.rgb = at<float>(ws, w.rgb);
  m.gocc = at<float>(ws, w.gocc);
  m.grgb = at<float>(ws, w.grgb);
  m.dpts = at<double>(ws, w.dpts);
  m.slab = at<float>(ws, w.slab);
  m.rec = w.save ? at<float>(ws, w.rec) : nullptr;
  m.cfeat = w.save ? m.rec : (w.fuse ? nullptr : at<float>(ws, w.feat));
  m.claim_rows = w.claims;  // only grids with a row map (nc_grid.grad_rows) claim
  if (w.claims) {
    m.claim_cnt = at<int32_t>(ws, w.claim_cnt);
    m.claim_tmp = at<int64_t>(ws, w.claim_tmp);
    m.claim_cap = w.claim_cap;
  }
  m.dfeat = w.det ? at<float>(ws, w.dfeat) : nullptr;
  m.range_flag = at<uint32_t>(ws, w.rflag);
  m.wimg = at<char>(ws, w.wimg);
  m.dximg = w.save ? at<float>(ws, w.dximg) : nullptr;
  m.bslab = w.save ? at<float>(ws, w.bslab) : nullptr;
  m.bslab_rows = w.bslab_rows;
  m.jac = w.has_jac ? at<float>(ws, w.jac) : nullptr;
}

// the weight-image builders of k_ray_setup / k_points_prep for k_mlp_fwd's jobs (nc_wimage.h)
static WImgCtx wimg_ctx(const MlpCtx& m) {
  WImgCtx wi;
  std::memset(&wi, 0, sizeof(wi));
  wi.n_jobs = m.n_jobs;
  wi.img = const_cast<char*>(m.wimg);
  wi.dximg = const_cast<float*>(m.dximg);  // a forward for a backward: k_mlp_dx's image too
  wi.wgs_per_job = WIMG_WGS * (m.dximg ? 2 : 1);
  for (int j = 0; j < m.n_jobs; ++j) {
    wi.kind[j] = m.jobs[j].kind;
    wi.dec[j] = m.dec[m.jobs[j].kind];
  }
  return wi;
}

DetBufs det_bufs(void* ws, const Ws& w) {
  DetBufs d;
  for (int b = 0; b < 2; ++b) {
    d.key[b] = at<uint64_t>(ws, w.dkey[b]);
    d.val[b] = at<uint32_t>(ws, w.dval[b]);
  }
  d.w = at<float>(ws, w.dw);
  d.part = at<float>(ws, w.dpart);
  d.temp = at<void>(ws, w.dtemp);
  d.temp_bytes = w.dtemp_bytes;
  d.vbits = w.vbits;
  d.ppad = w.dppad;
  d.sort_bits = w.dsort_bits;
  return d;
}

// NC_DETERMINISTIC: voxel-index bits over the grids the stage's decoders sample
int stage_vbits(const Plan& pl, const nc_grid* grids) {
  uint64_t most = 1;
  for (int j = 0; j < pl.n_jobs; ++j) {
    const nc_grid& G = grids[pl.jobs[j].kind];
    const uint64_t v = (uint64_t)G.dims[0] * (uint64_t)G.dims[1] * (uint64_t)G.dims[2];
    if (v > most) most = v;
  }
  int b = 1;
  while ((uint64_t(1) << b) < most) ++b;
  return b;
}

// sparse gradient rows: does any decoder of the stage claim rows of its own grid?
bool stage_claims(const Plan& pl, const nc_grid* grids) {
  for (int j = 0; j < pl.n_jobs; ++j)
    if (grids[pl.jobs[j].kind].grad_rows) return true;
  return false;
}

// k_grid_gather with sparse-row claims: zero the shard counters, gather (claims),
// give the claims their rows (k_rows_compact)
// The forward's trilinear lookups run inside k_mlp_fwd (MlpCtx::fuse_gather) unless the
// forward also claims sparse gradient rows, saves the Jacobian, or a grid is not
// channels-last: then k_grid_gather runs first (and zero-fills the gradient buffer).
int gather_and_claim(MlpCtx& m, const Ws& w, hipStream_t s) {
  if (w.fuse) {  // (layout: stage_fuse, no claims, no Jacobian)
    m.fuse_gather = 1;
    return 0;
  }
  if (w.claims)
    if (int e = check_hip(hipMemsetAsync(m.claim_cnt, 0, (size_t)MAX_JOBS * CLAIM_SHARDS * 4, s), "claim counters"))
      return e;
  if (int e = check_hip(timed(KID_GRID_GATHER, s, [&] { return launch_grid_gather(m, s); }), "k_grid_gather")) return e;
  if (w.claims)
    if (int e = check_hip(timed(KID_ROWS_CLAIM, s, [&] { return launch_rows_compact(m, s); }), "k_rows_compact"))
      return e;
  return 0;
}

// NC_LOSS_MAPPER forward for a backward: compositing, loss terms and the compositing
// backward for d loss = 1 in one kernel (k_composite_fwd_loss; NICECORE_FUSED_LOSS=0 for
// the three-kernel path).  Both sum the loss in a fixed order; NC_DETERMINISTIC keeps the
// three-kernel path (k_loss's value, the reference's expression order).
// The fused mapper forward's gradient zero fill: -1 = at k_mlp_fwd's tail, else the
// percentage filled by k_ray_setup's extra workgroups (the rest by k_composite_fwd_loss's).
// NICECORE_FILL_SETUP_PCT=<0..100> or "fwd" (A/B).
static int fill_setup_pct() {
  static int pct = -2;
  if (pct == -2) {
    const char* e = std::getenv("NICECORE_FILL_SETUP_PCT");
    pct = 0;
    if (e && std::strcmp(e, "fwd") == 0) pct = -1;
    else if (e && *e) pct = std::max(0, std::min(100, std::atoi(e)));
  }
  return pct;
}

bool fused_mapper_loss(const nc_render_args* a) {
  static int on = -1;
  if (on < 0) {
    const char* e = std::getenv("NICECORE_FUSED_LOSS");
    on = (e && std::strcmp(e, "0") == 0) ? 0 : 1;
  }
  return on && a->loss == NC_LOSS_MAPPER && (a->flags & NC_SAVE_FOR_BACKWARD) && !(a->flags & NC_DETERMINISTIC);
}

int render_prepare(const nc_render_args* a, Plan& pl, Ws& w, int64_t& P, int& S) {
  if (!a) return fail(-1, "nicecore: args is NULL");
  if (a->abi_version != NC_ABI_VERSION) return fail(-2, "nicecore: ABI version mismatch");
  if (int e = plan_stage(a->stage, pl)) return e;
  if (a->n_rays < 0) return fail(-1, "nicecore: n_rays < 0");
  if (a->n_extra < 0 || (a->n_extra > 0 && !a->z_extra && a->n_rays > 0))
    return fail(-1, "nicecore: n_extra > 0 needs z_extra");
  if (a->n_strat < 1 || a->n_surf < 0 || a->n_surf > NC_MAX_SURF ||
      a->n_strat + a->n_surf + a->n_extra > NC_MAX_SAMPLES)
    return fail(-1, "nicecore: need 1 <= N_samples, 0 <= N_surface <= 32, N_samples + N_surface + n_extra <= 64");
  if (a->n_surf > 0 && !a->gt_depth && a->n_rays > 0) return fail(-1, "nicecore: N_surface > 0 requires gt_depth");
  if (a->stage == NC_STAGE_COARSE && a->gt_depth) return fail(-1, "nicecore: stage 'coarse' ignores gt_depth; pass NULL");
  S = a->n_strat + a->n_surf + a->n_extra;
  P = a->n_rays * S;
  if (a->flags & ~(NC_SAVE_FOR_BACKWARD | NC_DETERMINISTIC | NC_SAVE_POINT_JACOBIAN | NC_DEFER_PARAM_GRADS |
                   NC_NO_WEIGHT_GRAD_ALL))
    return fail(-1, "nicecore: unknown flags");
  if (a->loss < NC_LOSS_NONE || a->loss > NC_LOSS_TRACKER) return fail(-1, "nicecore: unknown loss " + std::to_string(a->loss));
  if (a->loss != NC_LOSS_NONE) {
    if (a->loss_flags & ~(NC_LOSS_COLOR | NC_LOSS_DYNAMIC)) return fail(-1, "nicecore: unknown loss_flags");
    if ((a->loss_flags & NC_LOSS_DYNAMIC) && a->loss != NC_LOSS_TRACKER)
      return fail(-1, "nicecore: NC_LOSS_DYNAMIC is the tracker's handle_dynamic");
    if (!a->loss_out || (a->n_rays > 0 && !a->loss_depth)) return fail(-1, "nicecore: the loss needs loss_depth and loss_out");
    if ((a->loss_flags & NC_LOSS_COLOR) && a->n_rays > 0 && !a->loss_color)
      return fail(-1, "nicecore: NC_LOSS_COLOR needs loss_color");
  } else if (a->loss_flags) {
    return fail(-1, "nicecore: loss_flags without a loss");
  }
  int vbits = -1;
  if (a->flags & NC_DETERMINISTIC) {
    vbits = stage_vbits(pl, a->grids);
    if (vbits > 60 || (int64_t)pl.n_jobs * det_ppad(P) * 8 >= (int64_t(1) << 32))
      return fail(-1, "nicecore: NC_DETERMINISTIC supports < 2^32 (job, point, corner) entries");
  }
  layout(a->n_rays, P, pl, true, (a->flags & NC_SAVE_FOR_BACKWARD) != 0, a->loss != NC_LOSS_NONE, w, vbits,
         (a->flags & NC_SAVE_POINT_JACOBIAN) != 0, stage_claims(pl, a->grids), stage_fuse(pl, a->grids),
         fused_mapper_loss(a));
  if (w.det && w.dtemp_bytes == 0) return fail(-1, "nicecore: radix-sort scratch size query failed");
  return 0;
}

void fill_ray(RayCtx& c, const nc_render_args* a, const Plan& pl, void* ws, const Ws& w, int64_t P, int S) {
  std::memset(&c, 0, sizeof(c));
  c.range_flag = at<uint32_t>(ws, w.rflag);
  c.lindisp = a->lindisp;
  c.t_rand = a->t_rand;
  c.N = a->n_rays;
  c.P = P;
  c.S = S;
  c.n_strat = a->n_strat;
  c.n_surf = a->n_surf;
  c.n_extra = a->n_extra;
  c.z_extra = a->z_extra;
  c.z_out = a->z_out;
  c.weights_out = a->weights_out;
  c.stage = a->stage;
  c.occ_a = pl.occ_a;
  c.occ_b = pl.occ_b;
  c.has_rgb = pl.has_rgb;
  c.n_jobs = pl.n_jobs;
  c.rays_o = a->rays_o;
  c.rays_d = a->rays_d;
  c.gt_depth = a->gt_depth;
  c.depth_max = a->depth_max ? a->depth_max : at<float>(ws, w.dmax);
  std::memcpy(c.bound, a->bound, sizeof(c.bound));
  std::memcpy(c.t_strat, a->t_strat, sizeof(c.t_strat));
  std::memcpy(c.t_surf, a->t_surf, sizeof(c.t_surf));
  c.z = at<double>(ws, w.z);
  c.pts = at<double>(ws, w.pts);
  c.xyz = at<float4>(ws, w.xyz);
  c.pf = at<float4>(ws, w.pf);
  for (int j = 0; j < pl.n_jobs; ++j) std::memcpy(c.job_bound[j], a->dec[pl.jobs[j].kind].bound, sizeof(c.job_bound[j]));
  c.occ = at<float>(ws, w.occ);
  c.rgb = at<float>(ws, w.rgb);
  c.depth = a->depth;
  c.var = a->var;
  c.color = a->color;
  c.g_depth = a->g_depth;
  c.g_var = a->g_var;
  c.g_color = a->g_color;
  c.gocc = at<float>(ws, w.gocc);
  c.grgb = at<float>(ws, w.grgb);
  c.dpts = at<double>(ws, w.dpts);
  c.g_rays_o = a->g_rays_o;
  c.g_rays_d = a->g_rays_d;
  c.loss = a->loss;
  c.loss_flags = a->loss_flags;
  c.w_color = (float)a->w_color;
  c.loss_depth = a->loss_depth;
  c.loss_color = a->loss_color;
  c.loss_out = a->loss_out;
  c.g_loss = a->g_loss;
  if (a->loss != NC_LOSS_NONE) {
    c.coef_d = at<double>(ws, w.coef_d);
    c.coef_c = at<float>(ws, w.coef_c);
  }
  c.valid = a->ray_valid;
  if (w.lcount) {
    c.loss_part = at<double>(ws, w.lpart);
    c.loss_count = at<unsigned>(ws, w.lcount);
  }
}

int fwd_grid_x(int64_t P, int n_jobs, int which) {
  const int64_t per = which == 0 ? FWD_THREADS / 64 * 16 * FWD_TILES : DX_THREADS / 64 * 16;
  const int64_t blocks = (P + per - 1) / per;
  int x = cu_count() * mlp_blocks_per_cu(which) / n_jobs;
  if (x < 1) x = 1;
  if (blocks < x) x = (int)(blocks > 0 ? blocks : 1);
  return x;
}

int64_t nparam_of(int kind) {
  switch (kind) {
    case K_COARSE: return Net<K_COARSE>::NPARAM;
    case K_MID: return Net<K_MID>::NPARAM;
    case K_FINE: return Net<K_FINE>::NPARAM;
    case K_COLOR: return Net<K_COLOR>::NPARAM;
  }
  return -1;
}

int reduce_params(const MlpCtx& m, const nc_decoder_params* dec, hipStream_t s, const RayCtx* rc);

// decoder backward: dX chains + trilinear backward (k_mlp_dx) -> weight gradients
// -> slab reduction
int mlp_backward(const MlpCtx& m, const nc_decoder_params* dec, int64_t P, hipStream_t s, const DetBufs* det,
                 const RayCtx* rc = nullptr, bool defer_params = false) {
  if (!m.rec) return fail(-1, "nicecore: backward needs a forward run with NC_SAVE_FOR_BACKWARD");
  const int dx_x = fwd_grid_x(P, m.n_jobs, 1);
  if (m.bslab && dx_x != m.bslab_rows) return fail(-1, "nicecore: k_mlp_dx grid differs from its workspace rows");
  bool vec = true;  // every grid k_mlp_dx reads is channels-last (device grid_vec_ok)
  for (int j = 0; j < m.n_jobs; ++j) vec = vec && host_vec_ok(m.grids[m.jobs[j].kind]);
  if (int e = check_hip(timed(KID_MLP_DX, s, [&] { return launch_mlp_dx(m, dx_x, vec, s); }), "k_mlp_dx")) return e;
  bool any_grid = false;
  for (int j = 0; j < m.n_jobs; ++j) any_grid |= m.jobs[j].need_grid != 0;
  if (m.dfeat && any_grid)
    if (int e = check_hip(timed(KID_DET_SCATTER, s, [&] { return launch_det_scatter(m, *det, s); }), "deterministic grid scatter")) return e;
  if (defer_params) {  // NC_DEFER_PARAM_GRADS: weight gradients later (nc_render_backward_params)
    if (!rc) return 0;
    return check_hip(timed(KID_RAY_GRADS, s, [&] { return launch_ray_grads(*rc, s); }), "k_ray_grads");
  }
  bool any_dw = false;
  for (int j = 0; j < m.n_jobs; ++j) any_dw |= m.jobs[j].need_dw != 0;
  if (any_dw)
    if (int e = check_hip(timed(KID_MLP_DW, s, [&] { return launch_mlp_dw(m, s); }), "k_mlp_dw")) return e;
  return reduce_params(m, dec, s, rc);
}

// slab reduction of the weight gradients; with rc, d rays_o / d rays_d in the same launch
int reduce_params(const MlpCtx& m, const nc_decoder_params* dec, hipStream_t s, const RayCtx* rc) {
  ParamReduceCtx r;
  std::memset(&r, 0, sizeof(r));
  r.n_jobs = m.n_jobs;
  r.slab_wgs = m.slab_wgs;
  r.slab_stride = m.slab_stride;
  r.slab = m.slab;
  std::memcpy(r.wg_off, m.dw_off, sizeof(r.wg_off));
  bool any = false;
  for (int j = 0; j < m.n_jobs; ++j) {
    r.jobs[j] = m.jobs[j];
    r.grad[j] = dec[m.jobs[j].kind].grad;
    r.nparam[j] = nparam_of(m.jobs[j].kind);
    any |= (r.grad[j] != nullptr);
  }
  if (!any) {
    if (!rc) return 0;
    return check_hip(timed(KID_RAY_GRADS, s, [&] { return launch_ray_grads(*rc, s); }), "k_ray_grads");
  }
  if (rc)
    return check_hip(timed(KID_PARAM_RAY, s, [&] { return launch_param_ray_reduce(r, max_param_count(), *rc, s); }),
                     "k_param_ray_reduce");
  return check_hip(timed(KID_PARAM_REDUCE, s, [&] { return launch_param_reduce(r, max_param_count(), s); }), "k_param_reduce");
}

}  // namespace

extern "C" {

int nc_abi_version(void) { return NC_ABI_VERSION; }

#ifndef NC_SRC_HASH
#define NC_SRC_HASH "unknown-source00"
#endif
// "nicecore-src-<hash>" is also found in the file's bytes (build.py:library_build_id)
static const char kBuildTag[] = "nicecore-src-" NC_SRC_HASH;
const char* nc_build_id(void) { return kBuildTag + 13; }

const char* nc_last_error(void) { return g_err.c_str(); }

int64_t nc_param_count(int decoder) { return nparam_of(decoder); }

int nc_timing_start(uint32_t kernel_mask) {
  for (auto& t : g_timing.used) g_timing.pool.push_back({t.b, t.e});
  g_timing.used.clear();
  g_timing.mask = kernel_mask;
  return 0;
}

int nc_timing_stop(double* total_ms, int64_t* launches, int max_kernels) {
  g_timing.mask = 0;
  for (int k = 0; k < max_kernels; ++k) {
    if (total_ms) total_ms[k] = 0.0;
    if (launches) launches[k] = 0;
  }
  for (auto& t : g_timing.used) {
    if (hipEventSynchronize(t.e) != hipSuccess) return fail(-4, "nc_timing_stop: event sync failed");
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, t.b, t.e);
    if (t.id < max_kernels) {
      if (total_ms) total_ms[t.id] += ms;
      if (launches) launches[t.id] += 1;
    }
    g_timing.pool.push_back({t.b, t.e});
  }
  g_timing.used.clear();
  return KID_COUNT;
}

const char* nc_kernel_name(int id) { return (id >= 0 && id < KID_COUNT) ? kKernelNames[id] : ""; }

int nc_profile_report(void) {
  if (!profile_on()) return 0;
  const int rc = prof_fold(g_prof.pending.size());
  int order[KID_COUNT];
  int n = 0;
  for (int k = 0; k < KID_COUNT; ++k)
    if (g_prof.launches[k] > 0) order[n++] = k;
  for (int a = 1; a < n; ++a)  // by total time, descending
    for (int b = a; b > 0 && g_prof.total_ms[order[b]] > g_prof.total_ms[order[b - 1]]; --b) {
      const int x = order[b];
      order[b] = order[b - 1];
      order[b - 1] = x;
    }
  double all = 0.0;
  for (int a = 0; a < n; ++a) all += g_prof.total_ms[order[a]];
  std::fprintf(stderr, "[NICE_CORE_PROFILE] per-kernel HIP-event times (launch stream)\n");
  std::fprintf(stderr, "  %-22s %10s %12s %10s %7s\n", "kernel", "launches", "total ms", "avg us", "share");
  for (int a = 0; a < n; ++a) {
    const int k = order[a];
    std::fprintf(stderr, "  %-22s %10lld %12.3f %10.2f %6.1f%%\n", kKernelNames[k], (long long)g_prof.launches[k],
                 g_prof.total_ms[k], 1e3 * g_prof.total_ms[k] / (double)g_prof.launches[k],
                 all > 0.0 ? 100.0 * g_prof.total_ms[k] / all : 0.0);
  }
  if (g_prof.captured)
    std::fprintf(stderr, "  (%lld launches enqueued during graph capture: replays not timed)\n",
                 (long long)g_prof.captured);
  return rc;
}

size_t nc_struct_size(int which) {
  switch (which) {
    case 0: return sizeof(nc_render_args);
    case 1: return sizeof(nc_points_args);
    case 2: return sizeof(nc_grid);
    case 3: return sizeof(nc_decoder_params);
    case 4: return sizeof(nc_sample_args);
    case 5: return sizeof(nc_frustum_args);
    case 6: return sizeof(nc_sparse_rows);
    case 7: return sizeof(nc_pdf_args);
    case 8: return sizeof(nc_adam_args);
    case 9: return sizeof(nc_adam_segment);
    case 10: return sizeof(nc_imap_render_args);
    case 11: return sizeof(nc_imap_points_args);
    case 12: return sizeof(nc_imap_params);
    case 13: return sizeof(nc_grid_rows_args);
  }
  return 0;
}

size_t nc_render_workspace_bytes(const nc_render_args* a) {
  Plan pl;
  Ws w;
  int64_t P;
  int S;
  if (render_prepare(a, pl, w, P, S)) return 0;
  return w.total;
}

int nc_render_forward(const nc_render_args* a, void* ws, size_t ws_bytes, void* stream) {
  Plan pl;
  Ws w;
  int64_t P;
  int S;
  if (int e = render_prepare(a, pl, w, P, S)) return e;
  if (int e = check_models(pl, a->grids, a->dec)) return e;
  if (ws_bytes < w.total || !ws) return fail(-1, "nicecore: workspace too small");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (a->n_rays == 0) {
    if (a->loss != NC_LOSS_NONE) return check_hip(hipMemsetAsync(a->loss_out, 0, sizeof(double), s), "loss memset");
    return 0;
  }
  if (!a->rays_o || !a->rays_d || !a->depth || !a->var || !a->color)
    return fail(-1, "nicecore: NULL ray input or output pointer");
  RayCtx rc;
  fill_ray(rc, a, pl, ws, w, P, S);
  rc.fuse_bwd = fused_mapper_loss(a);
  if (a->gt_depth && !a->depth_max) {
    if (a->n_rays <= kDmaxLocalRays) {
      rc.dmax_local = 1;  // reduced inside k_ray_setup
    } else if (int e = check_hip(timed(KID_DEPTH_MAX, s, [&] { return launch_depth_max(a->gt_depth, a->ray_valid, a->n_rays, at<float>(ws, w.dmax), s); }), "k_depth_max")) {
      return e;
    }
  }
  MlpCtx m;
  fill_mlp(m, P, pl, a->grids, a->dec, rc.pts, ws, w, false);
  for (int j = 0; j < m.n_jobs; ++j)  // NC_NO_WEIGHT_GRAD: no activation records for k_mlp_dw
    m.jobs[j].keep_h = (a->flags & NC_NO_WEIGHT_GRAD(m.jobs[j].kind)) ? 0 : 1;
  if (a->grad_zero && a->grad_zero_floats > 0) {  // the caller's gradient buffer, zeroed by the gather
    if ((reinterpret_cast<uintptr_t>(a->grad_zero) & 15) || (a->grad_zero_floats & 3))
      return fail(-1, "nicecore: grad_zero must be 16-byte aligned and a multiple of 4 floats");
    m.zero_fill = reinterpret_cast<float4*>(a->grad_zero);
    m.zero_n4 = a->grad_zero_floats / 4;
  }
  if (w.fuse && rc.fuse_bwd && m.zero_fill && fill_setup_pct() >= 0) {
    // zeroed on the CUs the per-ray kernels leave idle instead of at k_mlp_fwd's tail (a
    // serial tail: every workgroup of its one resident wave ends at once): the first
    // fill_setup_pct() percent by extra workgroups of k_ray_setup, the rest by extra
    // workgroups of k_composite_fwd_loss
    const int64_t nb = fused_loss_blocks(rc.N);
    rc.zero_fill = m.zero_fill;
    rc.zero_n4 = m.zero_n4;
    rc.zero_lo4 = (m.zero_n4 * fill_setup_pct() / 100 + 63) & ~int64_t(63);
    if (rc.zero_lo4 > rc.zero_n4) rc.zero_lo4 = rc.zero_n4;
#ifndef NC_FILL_WGS_PER_CU
#define NC_FILL_WGS_PER_CU 1
#endif
    rc.zero_wgs = (int32_t)std::max<int64_t>(64, NC_FILL_WGS_PER_CU * cu_count() - nb);
    rc.zero_wgs_setup = cu_count();
    m.zero_fill = nullptr;
    m.zero_n4 = 0;
  }
  if (int e = check_hip(timed(KID_RAY_SETUP, s, [&] { return launch_ray_setup(rc, wimg_ctx(m), s); }), "k_ray_setup")) return e;
  if (int e = gather_and_claim(m, w, s)) return e;
  if (!m.fuse_gather) {  // zeroed by k_grid_gather (else by k_mlp_fwd)
    m.zero_fill = nullptr;
    m.zero_n4 = 0;
  }
  if (int e = check_hip(timed(KID_MLP_FWD, s, [&] { return launch_mlp_fwd(m, s); }), "k_mlp_fwd")) return e;
  if (rc.fuse_bwd)
    return check_hip(timed(KID_COMPOSITE_FWD_LOSS, s, [&] { return launch_composite_fwd_loss(rc, s); }),
                     "k_composite_fwd_loss");
  if (int e = check_hip(timed(KID_COMPOSITE_FWD, s, [&] { return launch_composite_fwd(rc, s); }), "k_composite_fwd")) return e;
  if (a->loss != NC_LOSS_NONE)
    if (int e = check_hip(timed(KID_LOSS, s, [&] { return launch_loss(rc, s); }), "k_loss")) return e;
  return 0;
}

int nc_render_backward(const nc_render_args* a, void* ws, size_t ws_bytes, void* stream) {
  Plan pl;
  Ws w;
  int64_t P;
  int S;
  if (int e = render_prepare(a, pl, w, P, S)) return e;
  if (int e = check_models(pl, a->grids, a->dec)) return e;
  if (ws_bytes < w.total || !ws) return fail(-1, "nicecore: workspace too small");
  if (a->n_rays == 0) return 0;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  RayCtx rc;
  fill_ray(rc, a, pl, ws, w, P, S);
  const bool need_coord = a->g_rays_o || a->g_rays_d;
  MlpCtx m;
  fill_mlp(m, P, pl, a->grids, a->dec, rc.pts, ws, w, need_coord);
  for (int j = 0; j < m.n_jobs; ++j)
    if (m.jobs[j].need_dw && (a->flags & NC_NO_WEIGHT_GRAD(m.jobs[j].kind)))
      return fail(-1, "nicecore: a weight gradient was asked for a decoder flagged NC_NO_WEIGHT_GRAD");
  bool any = need_coord;
  for (int j = 0; j < m.n_jobs; ++j) any |= m.jobs[j].need_dw || m.jobs[j].need_grid;
  if (!any) return 0;
  // a fused mapper loss whose only upstream gradient is d loss: the forward's
  // k_composite_fwd_loss already wrote d raw for d loss = 1, k_mlp_dx scales by d loss
  if (fused_mapper_loss(a) && a->g_loss && !a->g_depth && !a->g_var && !a->g_color) {
    m.dout_scale = a->g_loss;
  } else {
    if (fused_mapper_loss(a)) {  // keep the forward's d raw for d loss = 1 (a retained graph's next
                                 // loss-only backward reads it): this backward's d raw goes elsewhere
      rc.gocc = at<float>(ws, w.gocc_b);
      rc.grgb = at<float>(ws, w.grgb_b);
      m.gocc = rc.gocc;
      m.grgb = rc.grgb;
    }
    if (int e = check_hip(timed(KID_COMPOSITE_BWD, s, [&] { return launch_composite_bwd(rc, s); }), "k_composite_bwd"))
      return e;
  }
  const DetBufs det = det_bufs(ws, w);
  return mlp_backward(m, a->dec, P, s, &det, need_coord ? &rc : nullptr,  // (+ ray grads, fused)
                      (a->flags & NC_DEFER_PARAM_GRADS) != 0);
}

int nc_render_backward_params(const nc_render_args* a, void* ws, size_t ws_bytes, void* stream) {
  Plan pl;
  Ws w;
  int64_t P;
  int S;
  if (int e = render_prepare(a, pl, w, P, S)) return e;
  if (int e = check_models(pl, a->grids, a->dec)) return e;
  if (ws_bytes < w.total || !ws) return fail(-1, "nicecore: workspace too small");
  if (a->n_rays == 0) return 0;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  RayCtx rc;
  fill_ray(rc, a, pl, ws, w, P, S);
  MlpCtx m;
  fill_mlp(m, P, pl, a->grids, a->dec, rc.pts, ws, w, false);
  for (int j = 0; j < m.n_jobs; ++j)
    if (m.jobs[j].need_dw && (a->flags & NC_NO_WEIGHT_GRAD(m.jobs[j].kind)))
      return fail(-1, "nicecore: a weight gradient was asked for a decoder flagged NC_NO_WEIGHT_GRAD");
  if (!m.rec) return fail(-1, "nicecore: backward needs a forward run with NC_SAVE_FOR_BACKWARD");
  bool any_dw = false;
  for (int j = 0; j < m.n_jobs; ++j) any_dw |= m.jobs[j].need_dw != 0;
  if (!any_dw) return 0;
  if (int e = check_hip(timed(KID_MLP_DW, s, [&] { return launch_mlp_dw(m, s); }), "k_mlp_dw")) return e;
  return reduce_params(m, a->dec, s, nullptr);
}

static int points_prepare(const nc_points_args* a, Plan& pl, Ws& w) {
  if (!a) return fail(-1, "nicecore: args is NULL");
  if (a->abi_version != NC_ABI_VERSION) return fail(-2, "nicecore: ABI version mismatch");
  if (int e = plan_stage(a->stage, pl)) return e;
  if (a->n_points < 0) return fail(-1, "nicecore: n_points < 0");
  if (a->flags & ~(NC_SAVE_FOR_BACKWARD | NC_DETERMINISTIC | NC_SAVE_POINT_JACOBIAN)) return fail(-1, "nicecore: unknown flags");
  int vbits = -1;
  if (a->flags & NC_DETERMINISTIC) {
    vbits = stage_vbits(pl, a->grids);
    if (vbits > 60 || (int64_t)pl.n_jobs * det_ppad(a->n_points) * 8 >= (int64_t(1) << 32))
      return fail(-1, "nicecore: NC_DETERMINISTIC supports < 2^32 (job, point, corner) entries");
  }
  layout(0, a->n_points, pl, false, (a->flags & NC_SAVE_FOR_BACKWARD) != 0, false, w, vbits,
         (a->flags & NC_SAVE_POINT_JACOBIAN) != 0, stage_claims(pl, a->grids), stage_fuse(pl, a->grids));
  if (w.det && w.dtemp_bytes == 0) return fail(-1, "nicecore: radix-sort scratch size query failed");
  return 0;
}

size_t nc_points_workspace_bytes(const nc_points_args* a) {
  Plan pl;
  Ws w;
  if (points_prepare(a, pl, w)) return 0;
  return w.total;
}

int nc_points_forward(const nc_points_args* a, void* ws, size_t ws_bytes, void* stream) {
  Plan pl;
  Ws w;
  if (int e = points_prepare(a, pl, w)) return e;
  if (int e = check_models(pl, a->grids, a->dec)) return e;
  if (ws_bytes < w.total || !ws) return fail(-1, "nicecore: workspace too small");
  if (a->n_points == 0) return 0;
  if (!a->pts || !a->raw) return fail(-1, "nicecore: NULL points input or raw output");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  MlpCtx m;
  fill_mlp(m, a->n_points, pl, a->grids, a->dec, a->pts, ws, w, false);
  if (int e = check_hip(launch_points_prep(m, wimg_ctx(m), (float4*)m.xyz, (float4*)m.pf, s), "k_points_prep")) return e;
  if (int e = gather_and_claim(m, w, s)) return e;
  if (int e = check_hip(timed(KID_MLP_FWD, s, [&] { return launch_mlp_fwd(m, s); }), "k_mlp_fwd")) return e;
  return check_hip(timed(KID_POINTS_ASSEMBLE, s, [&] { return launch_points_assemble(m, a->stage, a->raw, s); }), "k_points_assemble");
}

int nc_points_backward(const nc_points_args* a, void* ws, size_t ws_bytes, void* stream) {
  Plan pl;
  Ws w;
  if (int e = points_prepare(a, pl, w)) return e;
  if (int e = check_models(pl, a->grids, a->dec)) return e;
  if (ws_bytes < w.total || !ws) return fail(-1, "nicecore: workspace too small");
  if (a->n_points == 0) return 0;
  if (!a->pts || !a->g_raw) return fail(-1, "nicecore: NULL points input or upstream gradient");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  MlpCtx m;
  fill_mlp(m, a->n_points, pl, a->grids, a->dec, a->pts, ws, w, a->g_pts != nullptr);
  if (int e = check_hip(timed(KID_POINTS_SPLIT, s, [&] { return launch_points_split_grad(m, a->stage, a->g_raw, (float*)m.gocc, (float*)m.grgb, s); }), "k_points_split_grad"))
    return e;
  const DetBufs det = det_bufs(ws, w);
  if (int e = mlp_backward(m, a->dec, a->n_points, s, &det)) return e;
  if (a->g_pts)
    if (int e = check_hip(timed(KID_POINTS_GRADS, s, [&] { return launch_points_grads(m, a->g_pts, s); }), "k_points_grads")) return e;
  return 0;
}

static int sample_check(const nc_sample_args* a) {
  if (!a) return fail(-1, "nicecore: args is NULL");
  if (a->abi_version != NC_ABI_VERSION) return fail(-2, "nicecore: ABI version mismatch");
  if (a->pose_dtype != NC_POSE_F32 && a->pose_dtype != NC_POSE_F64) return fail(-1, "nicecore: unknown pose dtype");
  if (a->n_frames < 0 || a->n_per_frame < 0) return fail(-1, "nicecore: negative frame / ray count");
  if (a->H0 < 0 || a->W0 < 0 || a->H1 <= a->H0 || a->W1 <= a->W0) return fail(-1, "nicecore: empty sampling region");
  if (a->n_frames * a->n_per_frame > 0 && (!(a->c2w || a->cam) || (!a->indices && !(a->pix_i && a->pix_j))))
    return fail(-1, "nicecore: sampling needs c2w (or cam) and indices (or pix_i and pix_j)");
  if (a->c2w && a->cam) return fail(-1, "nicecore: pass c2w or cam, not both");
  if (a->pix_i && (a->depth || a->color)) return fail(-1, "nicecore: pix_i / pix_j rays gather no depth or colour");
  return 0;
}

int nc_sample_rays_forward(const nc_sample_args* a, void* stream) {
  if (int e = sample_check(a)) return e;
  if (a->n_frames * a->n_per_frame == 0) return 0;
  if (!a->rays_o || !a->rays_d) return fail(-1, "nicecore: NULL ray outputs");
  if ((a->depth && !a->gt_depth) || (a->color && !a->gt_color)) return fail(-1, "nicecore: NULL depth / colour output");
  if (a->inside && (!a->bound || !a->depth)) return fail(-1, "nicecore: the bbox pre-filter needs bound and depth");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  return check_hip(timed(KID_SAMPLE_RAYS, s, [&] { return launch_sample_rays(*a, s); }), "k_sample_rays");
}

int nc_sample_rays_backward(const nc_sample_args* a, void* stream) {
  if (int e = sample_check(a)) return e;
  if (a->n_frames == 0) return 0;
  if (!a->g_c2w && !(a->cam && a->g_cam)) return fail(-1, "nicecore: NULL pose gradient output");
  if (a->cam && !a->g_cam) return fail(-1, "nicecore: NULL camera-tensor gradient output");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  return check_hip(timed(KID_SAMPLE_POSE_GRAD, s, [&] { return launch_sample_pose_grad(*a, s); }), "k_sample_pose_grad");
}

int nc_grid_rows(const nc_grid_rows_args* a, void* stream) {
  if (!a) return fail(-1, "nicecore: args is NULL");
  if (a->abi_version != NC_ABI_VERSION) return fail(-2, "nicecore: ABI version mismatch");
  if (a->op != NC_ROWS_GATHER && a->op != NC_ROWS_SCATTER && a->op != NC_ROWS_ZERO)
    return fail(-1, "nicecore: nc_grid_rows: unknown op");
  if (a->n_rows < 0 || a->channels <= 0 || a->dims[0] <= 0 || a->dims[1] <= 0 || a->dims[2] <= 0)
    return fail(-1, "nicecore: nc_grid_rows: bad sizes");
  if (a->n_rows > 0 && (!a->rows || !a->grid || (a->op != NC_ROWS_ZERO && !a->packed)))
    return fail(-1, "nicecore: nc_grid_rows: NULL pointer");
  if (a->n_rows * a->channels >= (int64_t(1) << 40)) return fail(-1, "nicecore: nc_grid_rows: too many rows");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  return check_hip(timed(KID_GRID_ROWS, s, [&] { return launch_grid_rows(*a, s); }), "k_grid_rows");
}

int nc_frustum_mask(const nc_frustum_args* a, void* stream) {
  if (!a) return fail(-1, "nicecore: args is NULL");
  if (a->abi_version != NC_ABI_VERSION) return fail(-2, "nicecore: ABI version mismatch");
  if (a->nx < 0 || a->ny < 0 || a->nz < 0 || a->H < 1 || a->W < 1) return fail(-1, "nicecore: bad grid or image size");
  if (a->nx * a->ny * a->nz == 0) return 0;
  if (!a->xs || !a->ys || !a->zs || !a->depth || !a->mask || !a->scratch)
    return fail(-1, "nicecore: NULL frustum input or output");
  if (a->H > 32767 || a->W > 32767) return fail(-1, "nicecore: cv2.remap semantics need H, W < 32768");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  return check_hip(timed(KID_FRUSTUM, s, [&] { return launch_frustum_mask(*a, s); }), "k_frustum_mask");
}

int nc_sample_pdf(const nc_pdf_args* a, void* stream) {
  if (!a) return fail(-1, "nicecore: args is NULL");
  if (a->abi_version != NC_ABI_VERSION) return fail(-2, "nicecore: ABI version mismatch");
  if (a->n_rays < 0) return fail(-1, "nicecore: n_rays < 0");
  if (a->n_bins < 2 || a->n_bins > NC_MAX_SAMPLES || a->n_samples < 1 || a->n_samples > NC_MAX_SAMPLES)
    return fail(-1, "nicecore: sample_pdf needs 2 <= n_bins <= 64 and 1 <= n_samples <= 64");
  if (a->n_rays == 0) return 0;
  if (!a->bins || !a->weights || !a->samples || (!a->det && !a->u))
    return fail(-1, "nicecore: NULL bins, weights, samples or (det = 0) u");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  return check_hip(timed(KID_SAMPLE_PDF, s, [&] { return launch_sample_pdf(*a, s); }), "k_sample_pdf");
}

int nc_adam_step(const nc_adam_args* a, void* stream) {
  if (!a) return fail(-1, "nicecore: args is NULL");
  if (a->abi_version != NC_ABI_VERSION) return fail(-2, "nicecore: ABI version mismatch");
  if (!(a->step >= 1.0)) return fail(-1, "nicecore: adam step count must be >= 1");
  if (!(a->beta1 >= 0.0 && a->beta1 < 1.0 && a->beta2 >= 0.0 && a->beta2 < 1.0 && a->eps >= 0.0 && a->lr >= 0.0))
    return fail(-1, "nicecore: adam needs 0 <= beta < 1, eps >= 0, lr >= 0");
  if (a->mode == NC_ADAM_DENSE) {
    if (a->n < 0) return fail(-1, "nicecore: adam n < 0");
    if (a->n > 0 && (!a->param || !a->grad || !a->exp_avg || !a->exp_avg_sq))
      return fail(-1, "nicecore: adam: NULL param, grad or moment");
  } else if (a->mode == NC_ADAM_SPARSE_ROWS) {
    if (a->row_capacity < 0) return fail(-1, "nicecore: adam row_capacity < 0");
    if (a->weight_decay != 0.0) return fail(-1, "nicecore: the sparse-rows rule (SparseAdam) has no weight_decay");
    if (!a->row_count || (a->row_capacity > 0 && (!a->param || !a->grad || !a->exp_avg || !a->exp_avg_sq ||
                                                    !a->row_voxel)))
      return fail(-1, "nicecore: adam: NULL param, rows, moment or row count");
    if (a->voxel_stride < 1 || a->channel_stride < 1) return fail(-1, "nicecore: adam: bad voxel/channel stride");
  } else {
    return fail(-1, "nicecore: unknown adam mode");
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  return check_hip(timed(KID_ADAM, s, [&] { return launch_adam(*a, s); }), "k_adam");
}

int nc_adam_step_multi(const nc_adam_args* a, const nc_adam_segment* segs, int32_t n, void* stream) {
  if (!a || (n > 0 && !segs)) return fail(-1, "nicecore: args or segments is NULL");
  if (a->abi_version != NC_ABI_VERSION) return fail(-2, "nicecore: ABI version mismatch");
  if (n < 0) return fail(-1, "nicecore: adam: negative segment count");
  if (!(a->beta1 >= 0.0 && a->beta1 < 1.0 && a->beta2 >= 0.0 && a->beta2 < 1.0 && a->eps >= 0.0))
    return fail(-1, "nicecore: adam needs 0 <= beta < 1, eps >= 0, lr >= 0");
  for (int i = 0; i < n; ++i) {
    const nc_adam_segment& g = segs[i];
    if (g.n < 0 || !(g.step_dev || g.step >= 1.0) || !(g.lr >= 0.0))
      return fail(-1, "nicecore: adam segment: bad n, step or lr");
    if (g.n > 0 && (!g.param || !g.grad || !g.exp_avg || !g.exp_avg_sq))
      return fail(-1, "nicecore: adam segment: NULL param, grad or moment");
  }
  if (n == 0) return 0;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  return check_hip(timed(KID_ADAM, s, [&] { return launch_adam_multi(*a, segs, n, s); }), "k_adam_multi");
}

static int rows_check(const nc_sparse_rows* r, const char* what) {
  if (!r) return fail(-1, std::string("nicecore: ") + what + " is NULL");
  if (r->capacity < 0 || r->n_voxels < 0) return fail(-1, std::string("nicecore: ") + what + ": negative size");
  if (!r->row_count || (r->capacity > 0 && (!r->grad_rows || !r->row_voxel)))
    return fail(-1, std::string("nicecore: ") + what + ": NULL map, row_voxel or row_count");
  if (r->capacity > INT32_MAX || r->n_voxels > INT32_MAX)
    return fail(-1, std::string("nicecore: ") + what + ": sparse rows need < 2^31 voxels and rows");
  return 0;
}

int nc_sparse_rows_clear(const nc_sparse_rows* r, void* stream) {
  if (int e = rows_check(r, "rows")) return e;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  return check_hip(timed(KID_ROWS_CLEAR, s, [&] { return launch_rows_clear(*r, s); }), "k_rows_clear");
}

size_t nc_sparse_merge_temp_bytes(int64_t n_keys, int64_t n_voxels) {
  if (n_keys < 0 || n_voxels < 0 || n_keys > INT32_MAX) return 0;
  return rows_merge_temp_bytes(n_keys, n_voxels);
}

int nc_sparse_rows_merge(const nc_sparse_rows* in, const nc_sparse_rows* out, const int64_t* all_voxel,
                         const int32_t* all_count, int32_t world, int64_t rank_capacity, void* temp,
                         size_t temp_bytes, void* stream) {
  if (int e = rows_check(in, "in")) return e;
  if (int e = rows_check(out, "out")) return e;
  if (in->grad_rows != out->grad_rows || in->n_voxels != out->n_voxels)
    return fail(-1, "nicecore: merge in / out must share one voxel -> row map");
  if (world < 1 || rank_capacity < 0 || (int64_t)world * rank_capacity > INT32_MAX)
    return fail(-1, "nicecore: merge needs world >= 1 and world * rank_capacity < 2^31");
  if (in->row_voxel == out->row_voxel || (in->values && in->values == out->values))
    return fail(-1, "nicecore: merge writes new rows: out buffers must differ from in");
  const int64_t n = (int64_t)world * rank_capacity;
  if (n > 0 && (!all_voxel || !all_count || !out->values || !in->values))
    return fail(-1, "nicecore: merge needs all_voxel, all_count and both value buffers");
  if (n > 0 && (!temp || temp_bytes < nc_sparse_merge_temp_bytes(n, in->n_voxels)))
    return fail(-1, "nicecore: merge scratch too small (nc_sparse_merge_temp_bytes)");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  return check_hip(timed(KID_ROWS_MERGE, s, [&] {
                     return launch_rows_merge(*in, *out, all_voxel, all_count, world, rank_capacity, temp, temp_bytes, s);
                   }),
                   "sparse rows merge");
}

}  // extern "C"

// ---------------------------------------------------------------------------
// iMAP* (ABI v8): k_ray_setup -> [k_imap_embed -> 4 x k_imap_gemm (bias+ReLU) ->
// k_imap_gemm (output) -> k_imap_split] -> k_composite_fwd (volume density);
// backward: k_composite_bwd -> k_imap_dout -> 4 x k_imap_gemm (ReLU mask) ->
// k_imap_gemm (d emb) -> k_imap_fourier_bwd -> [dW: 6 split-K k_imap_gemm +
// bias column sums] -> [k_ray_grads].
// ---------------------------------------------------------------------------
namespace {

constexpr int IH = NC_IMAP_HIDDEN;
// flat parameter offsets, nn.Module.parameters() order of the iMAP* MLP: embedder._B,
// pts_linears[0..3].(weight, bias), output_linear.(weight, bias)
struct ImapOff {
  int64_t B = 0, w[4], b[4], wo, bo, total;
  ImapOff() {
    int64_t o = 3 * EMB;
    for (int l = 0; l < 4; ++l) {
      w[l] = o;
      o += (int64_t)IH * (l == 0 ? EMB : IH);
      b[l] = o;
      o += IH;
    }
    wo = o;
    o += 4 * IH;
    bo = o;
    total = o + 4;
  }
};

struct ImapWs {
  size_t dmax = 0, z = 0, pts = 0, pf = 0, emb = 0, h = 0, raw = 0, occ = 0, rgb = 0;
  size_t gocc = 0, grgb = 0, dout = 0, dz = 0, demb = 0, dx = 0, dpts = 0, gnorm = 0, wt = 0, total = 0;
  size_t wimg = 0, wflag = 0, wtimg = 0, wtflag = 0;  // split-f16 weight images (k_imap_wimage)
};

void imap_layout(int64_t N, int64_t P, bool rays, bool bwd, ImapWs& w) {
  size_t o = 0;
  auto take = [&](size_t& f, size_t bytes) { f = o; o = align256(o + bytes); };
  if (rays) {
    take(w.dmax, 4);
    take(w.z, (size_t)P * 8);
  }
  take(w.pts, rays ? (size_t)P * 24 : 0);
  take(w.pf, (size_t)P * 16);
  take(w.emb, (size_t)P * EMBP * 4);
  take(w.h, (size_t)4 * P * IH * 4);
  take(w.wimg, (size_t)3 * IH * imap_wimage_row(IH));  // W_1..3 images, forward B
  take(w.wflag, 16);
  take(w.raw, (size_t)P * 16);
  if (rays) {
    take(w.occ, (size_t)P * 4);
    take(w.rgb, (size_t)P * 12);
  }
  if (bwd) {
    if (rays) {
      take(w.gocc, (size_t)P * 4);
      take(w.grgb, (size_t)P * 12);
      take(w.gnorm, (size_t)N * 4);
      take(w.dout, (size_t)P * 16);
    }
    take(w.dz, (size_t)4 * P * IH * 4);
    take(w.demb, (size_t)P * EMBP * 4);
    take(w.dx, (size_t)P * EMBP * 4);
    take(w.dpts, (size_t)P * 24);
    take(w.wt, (size_t)(3 * IH + EMB) * IH * 4);  // W_1..3^T, W_0^T: the dX GEMMs' k-contiguous B
    take(w.wtimg, (size_t)(3 * IH + EMB) * imap_wimage_row(IH));  // and their split-f16 images
    take(w.wtflag, 16);
  }
  w.total = o;
}

int check_imap_params(const nc_imap_params& d, bool need_grad) {
  if (!d.fourier_B || !d.out_w || !d.out_b) return fail(-1, "nicecore: iMAP* parameter pointer is NULL");
  for (int l = 0; l < 4; ++l)
    if (!d.lin_w[l] || !d.lin_b[l]) return fail(-1, "nicecore: iMAP* parameter pointer is NULL");
  (void)need_grad;
  return 0;
}

ImapGemm gemm(const float* A, int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc, int64_t M, int64_t N,
              int64_t K) {
  ImapGemm g;
  std::memset(&g, 0, sizeof(g));
  g.A = A;
  g.B = B;
  g.C = C;
  g.lda = lda;
  g.ldb = ldb;
  g.ldc = ldc;
  g.M = M;
  g.N = N;
  g.K = K;
  return g;
}

int run_gemm(const ImapGemm& g, bool a_km, bool b_kn, hipStream_t s) {
  return check_hip(timed(KID_IMAP_GEMM, s, [&] { return launch_imap_gemm(g, a_km, b_kn, s); }), "k_imap_gemm");
}

// forward MLP over P points whose p.float() is in ws.pf: emb, h_0..h_3, raw
int imap_mlp_forward(const nc_imap_params& d, int64_t P, void* ws, const ImapWs& w, float* raw, hipStream_t s) {
  const float4* pf = at<float4>(ws, w.pf);
  float* emb = at<float>(ws, w.emb);
  float* h = at<float>(ws, w.h);
  if (int e = check_hip(timed(KID_IMAP_FOURIER, s, [&] { return launch_imap_embed(pf, d.fourier_B, P, emb, s); }),
                        "k_imap_embed"))
    return e;
  // W_1..3 split once per call (k_imap_gemm_h then copies their tiles)
  unsigned char* wimg = at<unsigned char>(ws, w.wimg);
  uint32_t* wflag = at<uint32_t>(ws, w.wflag);
  const int64_t irow = imap_wimage_row(IH);
  {
    ImapWImage im;
    std::memset(&im, 0, sizeof(im));
    for (int z = 0; z < 3; ++z) {
      im.src[z] = d.lin_w[z + 1];
      im.img[z] = wimg + (int64_t)z * IH * irow;
      im.N[z] = IH;
      im.K[z] = IH;
      im.ld[z] = IH;
    }
    im.flag = wflag;
    if (int e = check_hip(launch_imap_wimage(im, 3, s), "k_imap_wimage")) return e;
  }
  for (int l = 0; l < 4; ++l) {
    const float* x = l == 0 ? emb : h + (int64_t)(l - 1) * P * IH;
    const int64_t K = l == 0 ? EMB : IH;
    ImapGemm g = gemm(x, l == 0 ? EMBP : IH, d.lin_w[l], K, h + (int64_t)l * P * IH, IH, P, IH, K);
    g.bias = d.lin_b[l];
    g.relu = 1;
    if (l > 0) {
      g.Bimg = wimg + (int64_t)(l - 1) * IH * irow;
      g.bflag = wflag + (l - 1);
      g.bimg_row = irow;
    }
    if (int e = run_gemm(g, false, false, s)) return e;
  }
  // output layer (N = 4): a streaming kernel, not a 64-wide MFMA tile
  return check_hip(timed(KID_IMAP_GEMM, s, [&] { return launch_imap_out(h + 3 * P * IH, d.out_w, d.out_b, P, raw, s); }),
                   "k_imap_out");
}

// backward from d raw [P][4] (dout): ReLU-masked dX chain, Fourier backward, and the
// weight gradients (overwritten into d.grad) when d.grad != NULL
int imap_mlp_backward(const nc_imap_params& d, int64_t P, void* ws, const ImapWs& w, const float* dout, double* dpts,
                      hipStream_t s) {
  const float4* pf = at<float4>(ws, w.pf);
  const float* emb = at<float>(ws, w.emb);
  const float* h = at<float>(ws, w.h);
  float* dz = at<float>(ws, w.dz);
  float* demb = at<float>(ws, w.demb);
  float* dx = d.grad ? at<float>(ws, w.dx) : nullptr;
  const int64_t PH = P * IH;
  // W_l^T [in][out] (k = out contiguous): the dX GEMMs below read B(k, n) = W_l[k][n] as
  // rows of W_l^T, the layout whose tiles load as float4 rows (k_imap_gemm_h)
  float* wt = at<float>(ws, w.wt);
  float* wtl[4] = {wt + 3 * (int64_t)IH * IH, wt, wt + (int64_t)IH * IH, wt + 2 * (int64_t)IH * IH};
  unsigned char* wtimg = at<unsigned char>(ws, w.wtimg);
  uint32_t* wtflag = at<uint32_t>(ws, w.wtflag);
  const int64_t irow = imap_wimage_row(IH);
  unsigned char* timg[4] = {wtimg + 3 * (int64_t)IH * irow, wtimg, wtimg + (int64_t)IH * irow,
                            wtimg + 2 * (int64_t)IH * irow};
  {  // W_l^T as f32 (the exact fallback's B) and as split-f16 images, one launch
    ImapWImage im;
    std::memset(&im, 0, sizeof(im));
    for (int l = 0; l < 4; ++l) {
      im.src[l] = d.lin_w[l];
      im.img[l] = timg[l];
      im.f32t[l] = wtl[l];
      im.N[l] = l == 0 ? EMB : IH;  // rows of W_l^T = inputs of layer l
      im.K[l] = IH;
      im.ld[l] = l == 0 ? EMB : IH;
      im.trans[l] = 1;
    }
    im.flag = wtflag;
    if (int e = check_hip(launch_imap_wimage(im, 4, s), "k_imap_wimage")) return e;
  }
  // dz_3 = (dout W_out) . [h_3 > 0] (K = 4): a streaming kernel
  if (int e = check_hip(timed(KID_IMAP_GEMM, s, [&] { return launch_imap_out_bwd(dout, d.out_w, h + 3 * PH, P, dz + 3 * PH, s); }),
                        "k_imap_out_bwd"))
    return e;
  for (int l = 3; l >= 1; --l) {  // dz_{l-1} = (dz_l W_l) . [h_{l-1} > 0]
    ImapGemm g = gemm(dz + l * PH, IH, wtl[l], IH, dz + (l - 1) * PH, IH, P, IH, IH);
    g.mask = h + (l - 1) * PH;
    g.ldm = IH;
    g.Bimg = timg[l];
    g.bflag = wtflag + l;
    g.bimg_row = irow;
    if (int e = run_gemm(g, false, false, s)) return e;
  }
  if (dpts || dx) {
    ImapGemm g = gemm(dz, IH, wtl[0], IH, demb, EMBP, P, EMB, IH);  // d emb = dz_0 W_0
    g.Bimg = timg[0];
    g.bflag = wtflag;
    g.bimg_row = irow;
    if (int e = run_gemm(g, false, false, s)) return e;
    if (int e = check_hip(timed(KID_IMAP_FOURIER, s, [&] {
                            return launch_imap_fourier_bwd(pf, d.fourier_B, P, demb, dx, dpts, s);
                          }),
                          "k_imap_fourier_bwd"))
      return e;
  }
  if (!d.grad) return 0;
  const ImapOff off;
  if (int e = check_hip(hipMemsetAsync(d.grad, 0, (size_t)off.total * 4, s), "grad memset")) return e;
  float* G = d.grad;
  auto dw = [&](const float* A, int64_t lda, int64_t M, const float* B, int64_t ldb, int64_t N, float* C) {
    ImapGemm g = gemm(A, lda, B, ldb, C, N, M, N, P);
    g.atomic = 1;
    return run_gemm(g, true, true, s);
  };
  if (int e = dw(dout, 4, 4, h + 3 * PH, IH, IH, G + off.wo)) return e;                    // dW_out = dout^T h_3
  for (int l = 3; l >= 1; --l)
    if (int e = dw(dz + l * PH, IH, IH, h + (l - 1) * PH, IH, IH, G + off.w[l])) return e;  // dW_l = dz_l^T h_{l-1}
  if (int e = dw(dz, IH, IH, emb, EMBP, EMB, G + off.w[0])) return e;                       // dW_0 = dz_0^T emb
  if (int e = dw(reinterpret_cast<const float*>(pf), 4, 3, dx, EMBP, EMB, G + off.B)) return e;  // dB = pf^T dx
  if (int e = check_hip(launch_imap_colsum(dout, P, 4, 4, G + off.bo, s), "k_imap_colsum")) return e;
  for (int l = 0; l < 4; ++l)
    if (int e = check_hip(launch_imap_colsum(dz + l * PH, P, IH, IH, G + off.b[l], s), "k_imap_colsum")) return e;
  return 0;
}

int imap_render_prepare(const nc_imap_render_args* a, ImapWs& w, int64_t& P, int& S) {
  if (!a) return fail(-1, "nicecore: args is NULL");
  if (a->abi_version != NC_ABI_VERSION) return fail(-2, "nicecore: ABI version mismatch");
  if (a->n_rays < 0) return fail(-1, "nicecore: n_rays < 0");
  if (a->flags & ~NC_SAVE_FOR_BACKWARD) return fail(-1, "nicecore: unknown flags");
  if (a->n_extra < 0 || (a->n_extra > 0 && !a->z_extra && a->n_rays > 0))
    return fail(-1, "nicecore: n_extra > 0 needs z_extra");
  if (a->n_strat < 1 || a->n_strat + a->n_extra > NC_MAX_SAMPLES)
    return fail(-1, "nicecore: need 1 <= N_samples, N_samples + n_extra <= 64");
  S = a->n_strat + a->n_extra;
  P = a->n_rays * S;
  imap_layout(a->n_rays, P, true, (a->flags & NC_SAVE_FOR_BACKWARD) != 0, w);
  return 0;
}

void imap_fill_ray(RayCtx& c, const nc_imap_render_args* a, void* ws, const ImapWs& w, int64_t P, int S) {
  std::memset(&c, 0, sizeof(c));
  c.N = a->n_rays;
  c.P = P;
  c.S = S;
  c.n_strat = a->n_strat;
  c.n_surf = 0;
  c.n_extra = a->n_extra;
  c.z_extra = a->z_extra;
  c.z_out = a->z_out;
  c.weights_out = a->weights_out;
  c.stage = NC_STAGE_COLOR;
  c.occ_a = 0;
  c.occ_b = -1;
  c.has_rgb = 1;
  c.n_jobs = 0;
  c.rays_o = a->rays_o;
  c.rays_d = a->rays_d;
  c.gt_depth = a->gt_depth;
  c.depth_max = a->depth_max ? a->depth_max : at<float>(ws, w.dmax);
  std::memcpy(c.bound, a->bound, sizeof(c.bound));
  std::memcpy(c.t_strat, a->t_strat, sizeof(c.t_strat));
  c.z = at<double>(ws, w.z);
  c.pts = at<double>(ws, w.pts);
  c.pf = at<float4>(ws, w.pf);
  c.occ = at<float>(ws, w.occ);
  c.rgb = at<float>(ws, w.rgb);
  c.depth = a->depth;
  c.var = a->var;
  c.color = a->color;
  c.g_depth = a->g_depth;
  c.g_var = a->g_var;
  c.g_color = a->g_color;
  c.g_rays_o = a->g_rays_o;
  c.g_rays_d = a->g_rays_d;
  c.density = 1;
  if (w.gocc || w.dout) {
    c.gocc = at<float>(ws, w.gocc);
    c.grgb = at<float>(ws, w.grgb);
    c.gnorm = at<float>(ws, w.gnorm);
    c.dpts = at<double>(ws, w.dpts);
  }
}

int imap_points_prepare(const nc_imap_points_args* a, ImapWs& w) {
  if (!a) return fail(-1, "nicecore: args is NULL");
  if (a->abi_version != NC_ABI_VERSION) return fail(-2, "nicecore: ABI version mismatch");
  if (a->n_points < 0) return fail(-1, "nicecore: n_points < 0");
  if (a->flags & ~NC_SAVE_FOR_BACKWARD) return fail(-1, "nicecore: unknown flags");
  imap_layout(0, a->n_points, false, (a->flags & NC_SAVE_FOR_BACKWARD) != 0, w);
  return 0;
}

}  // namespace

extern "C" {

int64_t nc_imap_param_count(void) { return ImapOff().total; }

size_t nc_imap_render_workspace_bytes(const nc_imap_render_args* a) {
  ImapWs w;
  int64_t P;
  int S;
  if (imap_render_prepare(a, w, P, S)) return 0;
  return w.total;
}

int nc_imap_render_forward(const nc_imap_render_args* a, void* ws, size_t ws_bytes, void* stream) {
  ImapWs w;
  int64_t P;
  int S;
  if (int e = imap_render_prepare(a, w, P, S)) return e;
  if (int e = check_imap_params(a->dec, false)) return e;
  if (ws_bytes < w.total || !ws) return fail(-1, "nicecore: workspace too small");
  if (a->n_rays == 0) return 0;
  if (!a->rays_o || !a->rays_d || !a->depth || !a->var || !a->color)
    return fail(-1, "nicecore: NULL ray input or output pointer");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  RayCtx rc;
  imap_fill_ray(rc, a, ws, w, P, S);
  if (a->gt_depth && !a->depth_max) {
    if (a->n_rays <= kDmaxLocalRays) {
      rc.dmax_local = 1;
    } else if (int e = check_hip(timed(KID_DEPTH_MAX, s, [&] { return launch_depth_max(a->gt_depth, nullptr, a->n_rays, at<float>(ws, w.dmax), s); }), "k_depth_max")) {
      return e;
    }
  }
  WImgCtx no_img;  // iMAP*: no NICE decoder images
  std::memset(&no_img, 0, sizeof(no_img));
  if (int e = check_hip(timed(KID_RAY_SETUP, s, [&] { return launch_ray_setup(rc, no_img, s); }), "k_ray_setup")) return e;
  float* raw = at<float>(ws, w.raw);
  if (int e = imap_mlp_forward(a->dec, P, ws, w, raw, s)) return e;
  if (int e = check_hip(launch_imap_split(raw, P, at<float>(ws, w.occ), at<float>(ws, w.rgb), s), "k_imap_split"))
    return e;
  return check_hip(timed(KID_COMPOSITE_FWD, s, [&] { return launch_composite_fwd(rc, s); }), "k_composite_fwd");
}

int nc_imap_render_backward(const nc_imap_render_args* a, void* ws, size_t ws_bytes, void* stream) {
  ImapWs w;
  int64_t P;
  int S;
  if (int e = imap_render_prepare(a, w, P, S)) return e;
  if (int e = check_imap_params(a->dec, true)) return e;
  if (!(a->flags & NC_SAVE_FOR_BACKWARD)) return fail(-1, "nicecore: backward needs NC_SAVE_FOR_BACKWARD");
  if (ws_bytes < w.total || !ws) return fail(-1, "nicecore: workspace too small");
  if (a->n_rays == 0) return 0;
  const bool need_coord = a->g_rays_o || a->g_rays_d;
  if (!need_coord && !a->dec.grad) return 0;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  RayCtx rc;
  imap_fill_ray(rc, a, ws, w, P, S);
  if (int e = check_hip(timed(KID_COMPOSITE_BWD, s, [&] { return launch_composite_bwd(rc, s); }), "k_composite_bwd")) return e;
  float* dout = at<float>(ws, w.dout);
  if (int e = check_hip(launch_imap_dout(rc.gocc, rc.grgb, P, dout, s), "k_imap_dout")) return e;
  double* dpts = at<double>(ws, w.dpts);
  if (int e = imap_mlp_backward(a->dec, P, ws, w, dout, need_coord ? dpts : nullptr, s)) return e;
  if (!need_coord) return 0;
  rc.n_jobs = 1;  // the decoder's point gradients (one slot)
  return check_hip(timed(KID_RAY_GRADS, s, [&] { return launch_ray_grads(rc, s); }), "k_ray_grads");
}

int64_t nc_imap_points_activation_offset(const nc_imap_points_args* a, int layer) {
  ImapWs w;
  if (layer < 0 || layer > 3 || imap_points_prepare(a, w)) return -1;
  return (int64_t)(w.h + (size_t)layer * a->n_points * IH * 4);
}

size_t nc_imap_points_workspace_bytes(const nc_imap_points_args* a) {
  ImapWs w;
  if (imap_points_prepare(a, w)) return 0;
  return w.total;
}

int nc_imap_points_forward(const nc_imap_points_args* a, void* ws, size_t ws_bytes, void* stream) {
  ImapWs w;
  if (int e = imap_points_prepare(a, w)) return e;
  if (int e = check_imap_params(a->dec, false)) return e;
  if (ws_bytes < w.total || !ws) return fail(-1, "nicecore: workspace too small");
  if (a->n_points == 0) return 0;
  if (!a->pts || !a->raw) return fail(-1, "nicecore: NULL pts or raw");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (int e = check_hip(launch_imap_pf(a->pts, a->n_points, at<float4>(ws, w.pf), s), "k_imap_pf")) return e;
  return imap_mlp_forward(a->dec, a->n_points, ws, w, a->raw, s);
}

int nc_imap_points_backward(const nc_imap_points_args* a, void* ws, size_t ws_bytes, void* stream) {
  ImapWs w;
  if (int e = imap_points_prepare(a, w)) return e;
  if (int e = check_imap_params(a->dec, true)) return e;
  if (!(a->flags & NC_SAVE_FOR_BACKWARD)) return fail(-1, "nicecore: backward needs NC_SAVE_FOR_BACKWARD");
  if (ws_bytes < w.total || !ws) return fail(-1, "nicecore: workspace too small");
  if (a->n_points == 0) return 0;
  if (!a->g_raw) return fail(-1, "nicecore: NULL g_raw");
  if (!a->g_pts && !a->dec.grad) return 0;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  return imap_mlp_backward(a->dec, a->n_points, ws, w, a->g_raw, a->g_pts, s);
}

}  // extern "C"
