// abi_host_check.cpp -- the host side of libnicecore's C ABI under AddressSanitizer and
// UndefinedBehaviorSanitizer (SURVEY.md §5 "ASan on the host restatement"), no GPU needed.
//
// tools/asan/build.py compiles every csrc/*.hip with -Xarch_host -fsanitize=address and
// -Xarch_host -fsanitize=undefined (host code only; nothing here launches a kernel) and
// links this driver.  It walks the argument validation, the
// stage plans and the workspace layouts of every entry point -- the code paths that
// run on the host before any launch -- over the BASELINE configs' shapes and a set of
// malformed calls, and checks the documented results (0 / negative codes, error text,
// workspace sizes that grow with the batch).  Device pointers are fake, aligned,
// never dereferenced (the library only inspects them).
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>

#include "nicecore.h"

static int g_fail = 0;
#define EXPECT(c, what)                                                                     \
  do {                                                                                      \
    if (!(c)) {                                                                             \
      std::fprintf(stderr, "FAIL %s:%d %s (last error: %s)\n", __FILE__, __LINE__, what,    \
                   nc_last_error());                                                        \
      ++g_fail;                                                                             \
    }                                                                                       \
  } while (0)

static const float* fake_f(uintptr_t k) { return reinterpret_cast<const float*>(0x10000000ull + (k << 12)); }

static void fill_grid(nc_grid& g, int64_t D, int64_t H, int64_t W, uintptr_t k, bool channels_last, bool grad) {
  std::memset(&g, 0, sizeof(g));
  g.data = fake_f(k);
  g.grad = grad ? const_cast<float*>(fake_f(k + 100)) : nullptr;
  g.dims[0] = D;
  g.dims[1] = H;
  g.dims[2] = W;
  if (channels_last) {
    g.stride[0] = 1;
    g.stride[1] = H * W * 32;
    g.stride[2] = W * 32;
    g.stride[3] = 32;
  } else {
    g.stride[0] = D * H * W;
    g.stride[1] = H * W;
    g.stride[2] = W;
    g.stride[3] = 1;
  }
  std::memcpy(g.grad_stride, g.stride, sizeof(g.stride));
}

static void fill_dec(nc_decoder_params& d, int kind, uintptr_t k, bool grad) {
  std::memset(&d, 0, sizeof(d));
  for (int i = 0; i < 5; ++i) {
    if (kind != NC_DEC_COARSE) {
      d.fc_w[i] = fake_f(k + 2 * i);
      d.fc_b[i] = fake_f(k + 2 * i + 1);
    }
    d.lin_w[i] = fake_f(k + 20 + 2 * i);
    d.lin_b[i] = fake_f(k + 21 + 2 * i);
  }
  if (kind != NC_DEC_COARSE) d.fourier_B = fake_f(k + 40);
  d.out_w = fake_f(k + 41);
  d.out_b = fake_f(k + 42);
  d.grad = grad ? const_cast<float*>(fake_f(k + 43)) : nullptr;
  const double b[3][2] = {{-2.9, 8.94}, {-3.2, 5.76}, {-3.5, 3.54}};  // Replica room0, snapped
  const double m = kind == NC_DEC_COARSE ? 2.0 : 1.0;
  for (int a = 0; a < 3; ++a)
    for (int s = 0; s < 2; ++s) d.bound[a][s] = m * b[a][s];
}

static nc_render_args render_args(int stage, int64_t n, int n_surf, bool grads, bool cl) {
  nc_render_args a;
  std::memset(&a, 0, sizeof(a));
  a.abi_version = NC_ABI_VERSION;
  a.stage = stage;
  a.n_rays = n;
  a.n_strat = 32;
  a.n_surf = n_surf;
  a.flags = grads ? NC_SAVE_FOR_BACKWARD : 0;
  a.rays_o = fake_f(1);
  a.rays_d = fake_f(2);
  a.gt_depth = n_surf > 0 ? fake_f(3) : nullptr;
  const double b[3][2] = {{-2.9, 8.94}, {-3.2, 5.76}, {-3.5, 3.54}};
  std::memcpy(a.bound, b, sizeof(b));
  for (int i = 0; i < 32; ++i) a.t_strat[i] = (float)i / 31.f;
  for (int i = 0; i < n_surf; ++i) a.t_surf[i] = (double)i / (n_surf - 1);
  fill_grid(a.grids[NC_DEC_COARSE], 7, 8, 11, 10, cl, grads);
  fill_grid(a.grids[NC_DEC_MIDDLE], 21, 28, 37, 11, cl, grads);
  fill_grid(a.grids[NC_DEC_FINE], 43, 56, 74, 12, cl, grads);
  fill_grid(a.grids[NC_DEC_COLOR], 43, 56, 74, 13, cl, grads);
  for (int k = 0; k < 4; ++k) fill_dec(a.dec[k], k, 200 + 100 * k, grads);
  a.depth = reinterpret_cast<double*>(const_cast<float*>(fake_f(4)));
  a.var = reinterpret_cast<double*>(const_cast<float*>(fake_f(5)));
  a.color = const_cast<float*>(fake_f(6));
  return a;
}

int main() {
  EXPECT(nc_abi_version() == NC_ABI_VERSION, "abi version");
  for (int i = 0; i <= 13; ++i) EXPECT(nc_struct_size(i) > 0, "struct size");
  EXPECT(nc_struct_size(99) == 0, "unknown struct id");
  int64_t total = 0;
  for (int k = 0; k < 4; ++k) total += nc_param_count(k);
  EXPECT(total == 58956, "parameter count over the four decoders");
  EXPECT(nc_param_count(9) < 0, "unknown decoder");
  EXPECT(nc_imap_param_count() == 222747, "iMAP* parameter count");
  EXPECT(std::string(nc_kernel_name(1)) == "k_ray_setup", "kernel name");
  EXPECT(std::string(nc_kernel_name(-1)).empty() && std::string(nc_kernel_name(1000)).empty(), "bad kernel id");
  EXPECT(nc_profile_report() == 0, "profile report with the flag off");
  EXPECT(nc_timing_start(0xffffffffu) == 0, "timing start");
  EXPECT(nc_timing_stop(nullptr, nullptr, 0) >= 0, "timing stop (nothing recorded)");

  // ---- render: every stage, the BASELINE batch sizes, both layouts, with / without grads
  const int64_t sizes[] = {1, 200, 1000, 5000, 16384};
  for (int stage = 0; stage < 4; ++stage)
    for (int64_t n : sizes)
      for (int grads = 0; grads < 2; ++grads)
        for (int cl = 0; cl < 2; ++cl) {
          const int ns = stage == NC_STAGE_COARSE ? 0 : 16;
          nc_render_args a = render_args(stage, n, ns, grads, cl);
          const size_t w1 = nc_render_workspace_bytes(&a);
          EXPECT(w1 > 0, "render workspace");
          a.n_rays = 2 * n;
          EXPECT(nc_render_workspace_bytes(&a) > w1, "workspace grows with the batch");
          a.n_rays = n;
          if (grads) {
            a.flags |= NC_DETERMINISTIC;
            EXPECT(nc_render_workspace_bytes(&a) > w1, "NC_DETERMINISTIC adds its sort buffers");
            a.flags = NC_SAVE_FOR_BACKWARD | NC_SAVE_POINT_JACOBIAN;
            EXPECT(nc_render_workspace_bytes(&a) > w1, "NC_SAVE_POINT_JACOBIAN adds the Jacobian");
            a.flags = NC_SAVE_FOR_BACKWARD;
            a.loss = NC_LOSS_MAPPER;
            a.loss_flags = NC_LOSS_COLOR;
            a.loss_depth = fake_f(7);
            a.loss_color = fake_f(8);
            a.loss_out = reinterpret_cast<double*>(const_cast<float*>(fake_f(9)));
            EXPECT(nc_render_workspace_bytes(&a) > w1, "the fused loss adds its per-ray terms");
          }
          // too small a workspace is refused before anything is enqueued
          nc_render_args b = render_args(stage, n, ns, grads, cl);
          EXPECT(nc_render_forward(&b, reinterpret_cast<void*>(0x1000), 16, nullptr) == -1, "small workspace");
          EXPECT(nc_render_backward(&b, nullptr, 0, nullptr) == -1, "NULL workspace");
        }
  {  // empty batch: nothing to launch, success
    nc_render_args a = render_args(NC_STAGE_COLOR, 0, 16, true, true);
    const size_t w = nc_render_workspace_bytes(&a);
    EXPECT(w > 0, "empty-batch workspace");
    EXPECT(nc_render_forward(&a, reinterpret_cast<void*>(0x1000), w, nullptr) == 0, "empty forward");
    EXPECT(nc_render_backward(&a, reinterpret_cast<void*>(0x1000), w, nullptr) == 0, "empty backward");
  }
  {  // malformed render calls: negative codes, a message, no crash
    nc_render_args a = render_args(NC_STAGE_COLOR, 100, 16, true, true);
    nc_render_args b = a;
    b.abi_version = NC_ABI_VERSION - 1;
    EXPECT(nc_render_workspace_bytes(&b) == 0 && nc_render_forward(&b, nullptr, 0, nullptr) == -2, "ABI mismatch");
    b = a; b.stage = 7;
    EXPECT(nc_render_forward(&b, nullptr, 0, nullptr) < 0, "unknown stage");
    b = a; b.n_strat = 0;
    EXPECT(nc_render_workspace_bytes(&b) == 0, "n_strat 0");
    b = a; b.n_surf = 40;
    EXPECT(nc_render_workspace_bytes(&b) == 0, "n_surf > 32");
    b = a; b.n_strat = 60;
    EXPECT(nc_render_workspace_bytes(&b) == 0, "more than 64 samples");
    b = a; b.gt_depth = nullptr;
    EXPECT(nc_render_workspace_bytes(&b) == 0, "surface samples without gt_depth");
    b = a; b.stage = NC_STAGE_COARSE;
    EXPECT(nc_render_workspace_bytes(&b) == 0, "coarse stage with gt_depth");
    b = a; b.flags = 1 << 20;
    EXPECT(nc_render_workspace_bytes(&b) == 0, "unknown flags");
    b = a; b.loss = 9;
    EXPECT(nc_render_workspace_bytes(&b) == 0, "unknown loss");
    b = a; b.loss = NC_LOSS_MAPPER; b.loss_flags = NC_LOSS_DYNAMIC;
    b.loss_depth = fake_f(7); b.loss_out = reinterpret_cast<double*>(const_cast<float*>(fake_f(9)));
    EXPECT(nc_render_workspace_bytes(&b) == 0, "handle_dynamic on the mapper loss");
    b = a; b.loss_flags = NC_LOSS_COLOR;
    EXPECT(nc_render_workspace_bytes(&b) == 0, "loss flags without a loss");
    b = a; b.n_extra = 4;
    EXPECT(nc_render_workspace_bytes(&b) == 0, "n_extra without z_extra");
    b = a; b.n_rays = -1;
    EXPECT(nc_render_workspace_bytes(&b) == 0, "negative ray count");
    b = a; b.grids[NC_DEC_FINE].data = nullptr;
    const size_t w = nc_render_workspace_bytes(&a);
    EXPECT(nc_render_forward(&b, reinterpret_cast<void*>(0x1000), w, nullptr) < 0, "missing grid");
    b = a; b.grids[NC_DEC_MIDDLE].dims[1] = 0;
    EXPECT(nc_render_forward(&b, reinterpret_cast<void*>(0x1000), w, nullptr) < 0, "empty grid dimension");
    b = a; b.dec[NC_DEC_COLOR].lin_w[3] = nullptr;
    EXPECT(nc_render_forward(&b, reinterpret_cast<void*>(0x1000), w, nullptr) < 0, "missing decoder weight");
    b = a; b.rays_o = nullptr;
    EXPECT(nc_render_forward(&b, reinterpret_cast<void*>(0x1000), w, nullptr) < 0, "NULL rays");
    b = a; b.flags = NC_SAVE_FOR_BACKWARD | NC_NO_WEIGHT_GRAD(NC_DEC_COLOR);
    const size_t w2 = nc_render_workspace_bytes(&b);
    EXPECT(nc_render_backward(&b, reinterpret_cast<void*>(0x1000), w2, nullptr) < 0,
           "weight gradient of a decoder flagged NC_NO_WEIGHT_GRAD");
    EXPECT(std::strlen(nc_last_error()) > 0, "error text");
  }

  // ---- points (NICE.forward on caller points, Mesher chunks)
  for (int stage = 0; stage < 4; ++stage)
    for (int64_t P : {int64_t(0), int64_t(1), int64_t(48000), int64_t(500000)}) {
      nc_points_args p;
      std::memset(&p, 0, sizeof(p));
      p.abi_version = NC_ABI_VERSION;
      p.stage = stage;
      p.n_points = P;
      nc_render_args r = render_args(stage, 1, 0, true, true);
      std::memcpy(p.grids, r.grids, sizeof(p.grids));
      std::memcpy(p.dec, r.dec, sizeof(p.dec));
      EXPECT(nc_points_workspace_bytes(&p) > 0, "points workspace");
      p.flags = 1 << 12;
      EXPECT(nc_points_workspace_bytes(&p) == 0, "points: unknown flags");
      p.flags = 0;
      p.n_points = -5;
      EXPECT(nc_points_workspace_bytes(&p) == 0, "points: negative count");
    }

  // ---- the other entry points' argument checks
  {
    nc_sample_args s;
    std::memset(&s, 0, sizeof(s));
    s.abi_version = NC_ABI_VERSION;
    EXPECT(nc_sample_rays_forward(&s, nullptr) < 0, "sampling: empty region");
    s.H1 = 680; s.W1 = 1200; s.pose_dtype = 7;
    EXPECT(nc_sample_rays_forward(&s, nullptr) < 0, "sampling: unknown pose dtype");
    s.pose_dtype = NC_POSE_F32;
    s.n_frames = 1; s.n_per_frame = 200;
    EXPECT(nc_sample_rays_forward(&s, nullptr) < 0, "sampling: no c2w / indices");
    EXPECT(nc_sample_rays_backward(&s, nullptr) < 0, "pose gradient: no c2w");
    nc_grid_rows_args g;
    std::memset(&g, 0, sizeof(g));
    g.abi_version = NC_ABI_VERSION;
    g.op = 9;
    EXPECT(nc_grid_rows(&g, nullptr) < 0, "grid rows: unknown op");
    g.op = NC_ROWS_GATHER; g.n_rows = -1;
    EXPECT(nc_grid_rows(&g, nullptr) < 0, "grid rows: bad size");
    nc_frustum_args f;
    std::memset(&f, 0, sizeof(f));
    f.abi_version = NC_ABI_VERSION;
    EXPECT(nc_frustum_mask(&f, nullptr) < 0, "frustum: empty image");
    f.nx = f.ny = f.nz = 4;
    f.H = 40000; f.W = 10; f.xs = f.ys = f.zs = fake_f(1); f.depth = fake_f(2);
    f.mask = reinterpret_cast<uint8_t*>(const_cast<float*>(fake_f(3)));
    f.scratch = reinterpret_cast<uint32_t*>(const_cast<float*>(fake_f(4)));
    EXPECT(nc_frustum_mask(&f, nullptr) < 0, "frustum: image too large for cv2.remap");
    nc_pdf_args d;
    std::memset(&d, 0, sizeof(d));
    d.abi_version = NC_ABI_VERSION;
    d.n_bins = 1;
    EXPECT(nc_sample_pdf(&d, nullptr) < 0, "sample_pdf: one bin");
    nc_adam_args o;
    std::memset(&o, 0, sizeof(o));
    o.abi_version = NC_ABI_VERSION;
    EXPECT(nc_adam_step(&o, nullptr) < 0, "adam: step 0");
    o.step = 1; o.beta1 = 0.9; o.beta2 = 0.999; o.mode = 5;
    EXPECT(nc_adam_step(&o, nullptr) < 0, "adam: unknown mode");
    EXPECT(nc_adam_step_multi(&o, nullptr, 2, nullptr) < 0, "adam multi: NULL segments");
    nc_sparse_rows sr;
    std::memset(&sr, 0, sizeof(sr));
    sr.capacity = -1;
    EXPECT(nc_sparse_rows_clear(&sr, nullptr) < 0, "sparse rows: negative capacity");
    EXPECT(nc_sparse_rows_clear(nullptr, nullptr) < 0, "sparse rows: NULL");
    nc_imap_render_args ir;
    std::memset(&ir, 0, sizeof(ir));
    ir.abi_version = NC_ABI_VERSION;
    ir.n_rays = 5000;
    ir.n_strat = 32;
    EXPECT(nc_imap_render_workspace_bytes(&ir) > 0, "iMAP* workspace");
    ir.n_strat = 0;
    EXPECT(nc_imap_render_workspace_bytes(&ir) == 0, "iMAP*: n_strat 0");
  }
  std::fprintf(stderr, "abi_host_check: %s (%d failures)\n", g_fail ? "FAILED" : "ok", g_fail);
  return g_fail ? 1 : 0;
}
