"""The HIP path on the geometries of BASELINE.json configs[2..4] against the CPU oracle.

C3  ScanNet scene0000 (bound [[-2,11],[-2,11.5],[-2,5.5]] snapped; grids coarse [7,13,13],
    middle [23,42,40], fine = color [47,85,81]: non-power-of-two dims), 5000 rays:
      * stage color, S = 48, mapper/BA gradients (rays, three grids, all decoders);
      * the coarse mapper: stage coarse, no render depth (S = 32), coarse decoder on the
        2x bound (NICE_SLAM.py:208, Mapper.py:600);
      * the fused Mapper / Tracker loss at 5000 rays: the tracker's handle_dynamic median
        over more rays than k_loss's 4,096-key LDS cache (the uncached radix passes).
C4  Apartment, one 625-ray shard of a 5000-ray (40 keyframes x 125) window, rendered with
    the window's max(gt_depth) (Renderer.py:157/:194 batch-global max, fed by depth_max=);
    and two gloo ranks on this GPU, each one 625-ray half of a 1250-ray batch with the
    MAX pre-reduce and a SUM all-reduce of the gradients (the bench.py N > 1 exchange),
    equal to the single-process batch.
C5  the synthetic 10 x 10 x 3 m scene with its real grids: fine and color [271,867,867]
    (26.1 GB each), middle [135,433,433], generated in HBM:
      * 16,384 rays with sparse gradient rows (nicecore.sparse) vs the dense-gradient path
        on the same 26-GB grids: every row equals the dense gradient's row, nothing of the
        dense gradient lies outside the rows, and a cropped window of the rows scattered
        back equals that window of the dense gradient;
      * a 256-ray subset (one camera, a 32 x 32 pixel patch, depths <= 1 m) vs the oracle
        evaluated on windows of the grids around those rays (sample_grid_window: the
        lookups of F.grid_sample on the full grid, tests/test_oracle_window.py).

Scoring: the per-element gate of tests/test_gpu_elementwise.py (parity_common.
oracle_elementwise_gate): every element of every output and gradient within 4x the largest
error of three float32 oracles (plain and two unit-permuted) against the float64 truth,
plus 4x the float32 oracle's RMS error; grid gradients with the float32 oracle's support;
no gradient the reference does not produce.  Reference: src/utils/Renderer.py:95-262;
shapes from src/NICE_SLAM.py:243-320.
"""
import os
import subprocess
import sys

import pytest
import torch

from conftest import REPO
from parity_common import build_model, make_renderer, oracle_elementwise_gate, rel_err

KEYS = ("grid_middle", "grid_fine", "grid_color")


def scene_case(scene, n_rays, seed=7, grid_std=0.3):
    """Random-init decoders (occupancy biases lowered so rays see partial opacity) and
    N(0, grid_std) grids of the scene's shapes, synthetic rays."""
    from nicecore import decoder as D
    from nicecore import scene as S
    sc = S.make_scene(scene)
    gen = torch.Generator().manual_seed(seed)
    grids = S.init_grids(sc.shapes, generator=gen, std={k: grid_std for k in S.GRID_STD})
    m = D.build_default_nice(seed=seed)
    with torch.no_grad():
        m.middle_decoder.output_linear.bias.fill_(-0.5)
        m.fine_decoder.output_linear.bias.fill_(-0.4)
        m.coarse_decoder.output_linear.bias.fill_(-0.5)
    params = {k: v.detach().clone() for k, v in m.named_parameters()}
    ro, rd, dep, col = S.synth_rays(sc, n_rays, seed=seed + 1)
    return sc, grids, params, ro, rd, dep, col


def _upstream(n, seed=11):
    gen = torch.Generator().manual_seed(seed)
    return (torch.randn(n, generator=gen, dtype=torch.float64), torch.randn(n, generator=gen, dtype=torch.float64),
            torch.randn(n, 3, generator=gen))


def _hip_render(sc, grids, params, ro, rd, stage, gt, up, depth_max=None, sparse=False):
    model = build_model(params, sc.bound, sc.bound * 2, "cuda")
    ro_g, rd_g = ro.cuda().requires_grad_(True), rd.cuda().requires_grad_(True)
    g_g = {k: (v if v.is_cuda else v.cuda().contiguous(memory_format=torch.channels_last_3d)).requires_grad_(True)
           for k, v in grids.items()}
    sp = None
    if sparse:
        from nicecore.sparse import SparseGridGrads
        sp = SparseGridGrads(g_g, keys=KEYS)
    r = make_renderer(sc.bound)
    d_g, v_g, c_g = r.render_batch_ray(g_g, model, rd_g, ro_g, "cuda", stage, gt.cuda() if gt is not None else None,
                                       depth_max=depth_max.cuda() if depth_max is not None else None,
                                       sparse_grads=sp)
    torch.autograd.backward([d_g, v_g, c_g], [t.cuda() for t in up])
    got = {"depth": d_g.detach().cpu(), "var": v_g.detach().cpu(), "color": c_g.detach().cpu(),
           "grad/rays_o": ro_g.grad.cpu(), "grad/rays_d": rd_g.grad.cpu()}
    for k, v in g_g.items():
        if v.grad is not None:
            got["grad/" + k] = v.grad.cpu()
    for n, p in model.named_parameters():
        if p.grad is not None:
            got["grad/param/" + n] = p.grad.cpu()
    return got, sp, g_g


def _against_oracle(title, sc, grids, params, ro, rd, stage, gt, depth_max=None):
    cb = sc.bound * 2
    dec_b = {"coarse": cb, "middle": sc.bound, "fine": sc.bound, "color": sc.bound}
    up = _upstream(ro.shape[0])
    got, _, _ = _hip_render(sc, grids, params, ro, rd, stage, gt, up, depth_max=depth_max)
    bad = oracle_elementwise_gate(title, got, grids, params, dec_b, sc.bound, ro, rd, stage, gt, up,
                                  depth_max=depth_max)
    assert not bad, bad


# ----------------------------------------------------------------------------- C3 ScanNet

@pytest.mark.gpu
def test_c3_scannet_color_ba_5000_rays():
    sc, grids, params, ro, rd, dep, _ = scene_case("scannet_scene0000", 5000, seed=17)
    assert sc.shapes["grid_fine"] == [47, 85, 81] and sc.shapes["grid_coarse"] == [7, 13, 13]
    _against_oracle("C3 ScanNet color BA 5000", sc, grids, params, ro, rd, "color", dep)


@pytest.mark.gpu
def test_c3_scannet_coarse_mapper_5000_rays():
    """The coarse mapper (Mapper.py:600): stage coarse renders without depth (S = 32) and
    the coarse decoder normalises with the 2x bound; gradients to the coarse grid,
    the coarse decoder and the rays."""
    sc, grids, params, ro, rd, dep, _ = scene_case("scannet_scene0000", 5000, seed=19)
    _against_oracle("C3 ScanNet coarse 5000", sc, grids, params, ro, rd, "coarse", None)


@pytest.mark.gpu
@pytest.mark.parametrize("kind,color_term,dyn", [("tracker", True, True), ("mapper", True, False)])
def test_c3_scannet_fused_loss_5000_rays(kind, color_term, dyn):
    """k_loss at 5000 rays: the tracker's global lower median (handle_dynamic) is
    selected over more keys than the LDS cache holds."""
    from test_gpu_loss import _compare_fused_unfused
    sc, grids, params, ro, rd, dep, col = scene_case("scannet_scene0000", 5000, seed=23)
    model = build_model(params, sc.bound, sc.bound * 2, "cuda")
    g = {k: v.cuda().contiguous(memory_format=torch.channels_last_3d).requires_grad_(True) for k, v in grids.items()}
    _compare_fused_unfused(make_renderer(sc.bound), "color", model, g, ro.cuda().requires_grad_(True),
                           rd.cuda().requires_grad_(True), dep.cuda(), col.cuda(), kind, color_term, dyn)


# ----------------------------------------------------------------------------- C4 Apartment

@pytest.mark.gpu
def test_c4_apartment_625_ray_shard_of_5000_window():
    """One GPU's shard of C4: rays 625..1249 of a 5000-ray window, far clamp and
    zero-depth surface samples from the WINDOW's max(gt_depth)."""
    sc, grids, params, ro, rd, dep, _ = scene_case("apartment", 5000, seed=29)
    assert sc.shapes["grid_fine"] == [81, 53, 107]
    dmax = dep.max().reshape(1)
    sl = slice(625, 1250)
    assert float(dep[sl].max()) < float(dmax)  # the shard's own max differs: depth_max matters
    _against_oracle("C4 Apartment shard 625", sc, grids, params, ro[sl], rd[sl], "color", dep[sl], depth_max=dmax)


@pytest.mark.gpu
def test_c4_apartment_two_gloo_ranks_equal_full_batch(tmp_path):
    """Two ranks (gloo, one GPU) render 625-ray halves of a 1250-ray Apartment batch with
    the MAX pre-reduce of the depth bound and the SUM all-reduce of grid and decoder
    gradients: outputs and ray gradients equal the single-process batch's rows, the
    reduced gradients its gradients (float-atomic tolerance 1e-5 of max-abs)."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29641", HSA_ENABLE_IPC_MODE_LEGACY="0")
    procs = [subprocess.Popen([sys.executable, os.path.join(REPO, "tests", "shard_dist_worker.py"), str(tmp_path)],
                              env=dict(env, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r))) for r in range(2)]
    for p in procs:
        assert p.wait(timeout=110) == 0
    outs = [torch.load(tmp_path / f"shard_rank{r}.pt", weights_only=True) for r in range(2)]
    full = shard_full_batch()
    for k in ("depth", "var", "color", "grad/rays_o", "grad/rays_d"):
        got = torch.cat([outs[0][k], outs[1][k]])
        assert rel_err(got, full[k]) <= 1e-6, (k, rel_err(got, full[k]))
    for k, v in full.items():
        if k.startswith("grad/grid") or k.startswith("grad/param"):
            assert torch.equal(outs[0][k], outs[1][k]), k  # the all-reduced gradient agrees
            assert rel_err(outs[0][k], v) <= 1e-5, (k, rel_err(outs[0][k], v))


SHARD_RAYS = 1250


def shard_setup():
    sc, grids, params, ro, rd, dep, col = scene_case("apartment", SHARD_RAYS, seed=31)
    model = build_model(params, sc.bound, sc.bound * 2, "cuda")
    g = {k: v.cuda().contiguous(memory_format=torch.channels_last_3d).requires_grad_(True) for k, v in grids.items()}
    return sc, g, model, ro.cuda(), rd.cuda(), dep.cuda(), col.cuda()


def shard_step(sc, g, model, ro, rd, dep, col, depth_max):
    """render_batch_loss (Mapper loss, color stage) + backward on these rays."""
    ro_ = ro.detach().clone().requires_grad_(True)
    rd_ = rd.detach().clone().requires_grad_(True)
    r = make_renderer(sc.bound)
    d, u, c, L = r.render_batch_loss(g, model, rd_, ro_, "cuda", "color", dep, col, loss="mapper",
                                     w_color_loss=0.2, color_term=True, depth_max=depth_max)
    L.backward()
    return {"depth": d.detach(), "var": u.detach(), "color": c.detach(), "grad/rays_o": ro_.grad,
            "grad/rays_d": rd_.grad}


def shard_collect(out, g, model):
    for k, v in g.items():
        if v.grad is not None:
            out["grad/" + k] = v.grad
    for n, p in model.named_parameters():
        if p.grad is not None:
            out["grad/param/" + n] = p.grad
    return {k: v.detach().cpu() for k, v in out.items()}


def shard_full_batch():
    sc, g, model, ro, rd, dep, col = shard_setup()
    out = shard_step(sc, g, model, ro, rd, dep, col, dep.max().reshape(1))
    return shard_collect(out, g, model)


# ----------------------------------------------------------------------------- C5 200M voxels

def _c5_grids(dense_grads):
    import gc
    from nicecore import scene as S
    sc = S.make_scene("synthetic_c5")
    assert sc.shapes["grid_fine"] == [271, 867, 867] and sc.shapes["grid_color"] == [271, 867, 867]
    gc.collect()
    torch.cuda.empty_cache()  # an earlier C5 test's blocks stay in the caching allocator
    free, _ = torch.cuda.mem_get_info()
    need = S.grids_bytes({k: sc.shapes[k] for k in KEYS}) * (2 if dense_grads else 1) + (24 << 30)
    if free < need:
        pytest.skip(f"C5 needs {need >> 30} GiB of free HBM, {free >> 30} GiB free")
    shapes = {k: sc.shapes[k] for k in KEYS}
    grids = S.init_grids_device(shapes, seed=5, device="cuda", std={k: 0.3 for k in S.GRID_STD})
    return sc, grids


def _c5_params(seed=37):
    from nicecore import decoder as D
    m = D.build_default_nice(seed=seed)
    with torch.no_grad():
        m.middle_decoder.output_linear.bias.fill_(-0.5)
        m.fine_decoder.output_linear.bias.fill_(-0.4)
    return {k: v.detach().clone() for k, v in m.named_parameters()}


@pytest.mark.gpu
def test_c5_sparse_rows_equal_dense_on_26gb_grids():
    from nicecore import scene as S
    sc, grids = _c5_grids(dense_grads=True)
    params = _c5_params()
    ro, rd, dep, _ = S.synth_rays(sc, 16384, seed=41)
    up = _upstream(16384, seed=43)
    dense, _, g_g = _hip_render(sc, grids, params, ro, rd, "color", dep, up)
    dense_dev = {k: g_g[k].grad for k in KEYS}
    for v in g_g.values():
        v.grad = None
    sparse, sp, _ = _hip_render(sc, g_g, params, ro, rd, "color", dep, up, sparse=True)
    for k in ("depth", "var", "color"):
        assert torch.equal(sparse[k], dense[k]), k  # same forward
    for k in ("grad/rays_o", "grad/rays_d"):
        assert rel_err(sparse[k], dense[k]) <= 1e-6, k
    for k in dense:
        if k.startswith("grad/param"):
            assert rel_err(sparse[k], dense[k]) <= 1e-5, k
    for k in KEYS:
        D, H, W = sc.shapes[k]
        rows_dense = dense_dev[k].permute(0, 2, 3, 4, 1).reshape(-1, 32)  # channels-last view
        idx, vals = sp.indices(k), sp.values(k)
        assert idx.numel() > 100000 and torch.unique(idx).numel() == idx.numel(), k
        assert int(idx.max()) < D * H * W
        ref = rows_dense.index_select(0, idx)
        assert rel_err(vals, ref) <= 1e-5, (k, rel_err(vals, ref))
        # nothing of the dense gradient lies outside the rows
        tot = float(rows_dense.abs().sum(dtype=torch.float64))
        assert tot > 0 and float(ref.abs().sum(dtype=torch.float64)) == pytest.approx(tot, rel=1e-9), k
        # a 48 x 64 x 64 window around the densest rows, scattered back
        z, y, x = idx // (H * W), (idx // W) % H, idx % W
        z0 = int(z.median()) - 24
        y0, x0 = int(y.median()) - 32, int(x.median()) - 32
        z0, y0, x0 = max(z0, 0), max(y0, 0), max(x0, 0)
        inw = (z >= z0) & (z < z0 + 48) & (y >= y0) & (y < y0 + 64) & (x >= x0) & (x < x0 + 64)
        win = torch.zeros(48, 64, 64, 32, device="cuda")
        win[z[inw] - z0, y[inw] - y0, x[inw] - x0] = vals[inw]
        dwin = dense_dev[k][0, :, z0:z0 + 48, y0:y0 + 64, x0:x0 + 64].permute(1, 2, 3, 0)
        dwin = torch.nn.functional.pad(dwin, (0, 0, 0, 64 - dwin.shape[2], 0, 64 - dwin.shape[1], 0, 48 - dwin.shape[0]))
        assert int(inw.sum()) > 0, k
        assert rel_err(win, dwin) <= 1e-5, k


def _patch_rays(sc, n_side=16, seed=47):
    """One camera near the middle of the bound, an n_side x n_side pixel patch around the
    image centre (a narrow cone), gt_depth ~ U(0.3, 1.0) with every 10th ray at depth 0:
    every sample lies within 1.2 m of the camera, far from the bound (no clipped lookups)."""
    from nicecore.scene import _random_rotation
    gen = torch.Generator().manual_seed(seed)
    R = _random_rotation(gen)
    t = sc.bound[:, 0].float() + (sc.bound[:, 1] - sc.bound[:, 0]).float() * torch.tensor([0.45, 0.55, 0.5])
    i = sc.cx - n_side + 2 * n_side * torch.rand(n_side * n_side, generator=gen)
    j = sc.cy - n_side + 2 * n_side * torch.rand(n_side * n_side, generator=gen)
    dirs = torch.stack([(i - sc.cx) / sc.fx, -(j - sc.cy) / sc.fy, -torch.ones_like(i)], -1)
    rd = torch.sum(dirs[:, None, :] * R, -1).contiguous()
    ro = t.expand(rd.shape).contiguous()
    dep = 0.3 + 0.7 * torch.rand(rd.shape[0], generator=gen)
    dep[::10] = 0.0
    return ro, rd, dep


def _windows(sc, pts, grids_dev):
    """Per grid the index box of every trilinear corner of ``pts`` (+1 voxel), as a CPU
    copy of that window and its sample_grid_window spec."""
    lo, hi = sc.bound[:, 0], sc.bound[:, 1]
    win, spec = {}, {}
    for k in KEYS:
        D, H, W = sc.shapes[k]
        size = torch.tensor([W - 1, H - 1, D - 1], dtype=torch.float64)
        idx = (pts - lo) / (hi - lo) * size
        a = (idx.amin(0).floor() - 1).clamp_min(0).long()
        b = torch.minimum(idx.amax(0).ceil() + 1, size).long()
        (x0, y0, z0), (x1, y1, z1) = a.tolist(), b.tolist()
        win[k] = grids_dev[k][:, :, z0:z1 + 1, y0:y1 + 1, x0:x1 + 1].contiguous().cpu()
        spec[k] = ((D, H, W), (z0, y0, x0))
    return win, spec


@pytest.mark.gpu
def test_c5_256_rays_match_oracle_on_grid_windows():
    from oracle import nice_oracle as O
    sc, grids = _c5_grids(dense_grads=False)
    params = _c5_params(seed=53)
    ro, rd, dep = _patch_rays(sc)
    assert ro.shape[0] == 256
    _, pts = O.points_for_rays(ro, rd, sc.bound, dep, "color")
    pts = pts.reshape(-1, 3)
    lo, hi = sc.bound[:, 0], sc.bound[:, 1]
    assert bool(((pts > lo) & (pts < hi)).all())  # no masked or clipped samples
    win, spec = _windows(sc, pts, grids)
    assert sum(w.numel() for w in win.values()) * 4 < (1 << 30)  # windows, not 26-GB grids
    up = _upstream(256, seed=59)
    dec_b = {"coarse": sc.bound * 2, "middle": sc.bound, "fine": sc.bound, "color": sc.bound}
    got, sp, _ = _hip_render(sc, grids, params, ro, rd, "color", dep, up, sparse=True)
    for k in KEYS:  # the touched rows, scattered into the window's frame
        (D, H, W), (z0, y0, x0) = spec[k]
        idx, vals = sp.indices(k).cpu(), sp.values(k).cpu()
        z, y, x = idx // (H * W), (idx // W) % H, idx % W
        d, h, w = win[k].shape[2:]
        assert bool(((z >= z0) & (z < z0 + d) & (y >= y0) & (y < y0 + h) & (x >= x0) & (x < x0 + w)).all()), k
        dense = torch.zeros(d, h, w, 32)
        dense[z - z0, y - y0, x - x0] = vals
        got["grad/" + k] = dense.permute(3, 0, 1, 2).unsqueeze(0)
    with O.grid_windows(spec):
        bad = oracle_elementwise_gate("C5 256 rays on grid windows", got, win, params, dec_b, sc.bound, ro, rd,
                                      "color", dep, up)
    assert not bad, bad
