"""ORACLE — TEST INFRASTRUCTURE ONLY.  Never imported by the product path.

CPU restatement of NICE-SLAM's ``Renderer.render_batch_ray`` hot path, written
as plain functions over torch CPU ops with the reference's op sequence and
dtypes (float64 depth/coordinate chain, float32 features and decoders), so that
autograd through it yields the reference's gradients.  Used by

  * tests/ (parity checker for the HIP path, pinned against tests/golden/*.npz,
    which tests/golden/make_golden.py captured from the reference itself), and
  * bench.py's ``cpu_baseline`` leg (``kind: "port"``).

Parity status: PINNED — tests/test_oracle_golden.py checks this module against
the golden vectors produced by importing /root/reference in the build container.

Every function cites the reference lines it restates.
"""
from __future__ import annotations

import contextlib

import torch
import torch.nn.functional as F

# Compute dtype of the reference's float32 stages.  The reference is float32
# (FLOAT = torch.float32); tests switch it to float64 with ``float64_mode()`` to
# obtain a ground truth against which both fp32 implementations are scored.
FLOAT = torch.float32
# float64 mode with the reference's explicit input roundings kept: the lookup coordinates
# (decoder.py:182 ``vgrid = p_nor[:, :, None, None].float()``) and the Fourier input
# (``p.float()``) rounded to float32 first, everything after them in float64 -- the exact-
# arithmetic value of the reference's float32 program, the per-element truth of
# tests/test_gpu_elementwise.py.  Plain float64_mode() computes from the unrounded points.
ROUND32 = False


@contextlib.contextmanager
def float64_mode(round_inputs: bool = False):
    global FLOAT, ROUND32
    old, oldr = FLOAT, ROUND32
    FLOAT, ROUND32 = torch.float64, round_inputs
    try:
        yield
    finally:
        FLOAT, ROUND32 = old, oldr


def _in32(t: torch.Tensor) -> torch.Tensor:
    """An input the reference rounds to float32, in the compute dtype."""
    return t.to(torch.float32).to(FLOAT) if ROUND32 else t.to(FLOAT)

STAGE_DECODERS = {  # decoder.py:341-370 (which MLPs feed raw at each stage)
    "coarse": ("coarse",),
    "middle": ("middle",),
    "fine": ("fine", "middle"),
    "color": ("fine", "color", "middle"),
}


def normalize_3d_coordinate(p: torch.Tensor, bound: torch.Tensor) -> torch.Tensor:
    """common.py:280-295 — per axis ((p-lo)/(hi-lo))*2-1 in float64."""
    cols = [((p[:, k] - bound[k, 0]) / (bound[k, 1] - bound[k, 0])) * 2 - 1.0 for k in range(3)]
    return torch.stack(cols, dim=1)


# Windowed grids (tests of the 26-GB C5 grids only): grid key -> (full [D, H, W], window
# offset (z0, y0, x0)).  The grid tensor passed for such a key is a window
# grid[:, :, z0:z0+d, y0:y0+h, x0:x0+w] of a grid too large for the CPU, and its lookups
# are computed as F.grid_sample on the FULL grid would compute them (sample_grid_window).
_WINDOWS: dict = {}


@contextlib.contextmanager
def grid_windows(spec: dict):
    """Within the block, lookups of the grids named in ``spec`` use sample_grid_window."""
    global _WINDOWS
    old, _WINDOWS = _WINDOWS, dict(spec)
    try:
        yield
    finally:
        _WINDOWS = old


def sample_grid_window(p, window, bound, full_dims, offset):
    """F.grid_sample(grid, normalize(p), border, align_corners=True) of decoder.py:179-188
    for a grid of which only ``window`` is held, restating ATen's grid_sampler_3d (CPU):
    unnormalise on the FULL grid ix = ((x + 1) / 2) * (W - 1) in the compute dtype, clip
    to [0, W - 1] (border; zero coordinate gradient where clipped or on a border), corners floor(ix) and
    +1, weights tnw = (ix_bse - ix)(iy_bse - iy)(iz_bse - iz) ... bse, corners outside the
    grid skipped, out = tnw·v_tnw + tne·v_tne + tsw + tse + bnw + bne + bsw + bse in that
    order.  The window offset is subtracted from the integer corner indices only, so the
    weights are those of the full grid, bit for bit.  A corner outside the window that is
    inside the full grid raises (the caller sized the window too small).  Returns [P, C]."""
    vn = _in32(normalize_3d_coordinate(p, bound))
    D, H, W = full_dims
    z0, y0, x0 = offset
    d, h, w = window.shape[2:]
    src = window[0].permute(1, 2, 3, 0)  # [d, h, w, C]

    def unnorm(x, size):
        # clip_coordinates_set_grad: the borders count as clipped (zero gradient at 0
        # and at size - 1 exactly), unlike clamp's inclusive gradient
        u = ((x + 1) / 2) * (size - 1)
        keep = (u > 0) & (u < size - 1)
        return torch.where(keep, u, u.detach().clamp(0, size - 1))

    ix, iy, iz = unnorm(vn[:, 0], W), unnorm(vn[:, 1], H), unnorm(vn[:, 2], D)
    fx, fy, fz = ix.detach().floor(), iy.detach().floor(), iz.detach().floor()
    out = None
    # ATen's corner order: t/b = z, n/s = y, w/e = x
    for dz, dy, dx in ((0, 0, 0), (0, 0, 1), (0, 1, 0), (0, 1, 1), (1, 0, 0), (1, 0, 1), (1, 1, 0), (1, 1, 1)):
        cx, cy, cz = fx + dx, fy + dy, fz + dz
        # the weight of corner (dx, dy, dz) is built from the opposite corner's distances
        wx = (ix - fx) if dx else ((fx + 1) - ix)
        wy = (iy - fy) if dy else ((fy + 1) - iy)
        wz = (iz - fz) if dz else ((fz + 1) - iz)
        wgt = wx * wy * wz
        inb = (cx < W) & (cy < H) & (cz < D)
        lx, ly, lz = (cx - x0).long(), (cy - y0).long(), (cz - z0).long()
        inw = (lx >= 0) & (lx < w) & (ly >= 0) & (ly < h) & (lz >= 0) & (lz < d)
        if bool((inb & ~inw).any()):
            raise ValueError("sample_grid_window: a lookup needs a voxel outside the window")
        val = src[lz.clamp(0, d - 1), ly.clamp(0, h - 1), lx.clamp(0, w - 1)]  # [P, C]
        term = val * torch.where(inb, wgt, torch.zeros_like(wgt))[:, None]
        out = term if out is None else out + term
    return out


def sample_grid_feature(p: torch.Tensor, grid: torch.Tensor, bound: torch.Tensor, key: str = "") -> torch.Tensor:
    """decoder.py:179-188 — trilinear (mode 'bilinear' on 5-D), border padding,
    align_corners=True.  Returns [P, C]."""
    if key in _WINDOWS:
        return sample_grid_window(p, grid, bound, *_WINDOWS[key])
    vgrid = _in32(normalize_3d_coordinate(p, bound).unsqueeze(0)[:, :, None, None])
    c = F.grid_sample(grid, vgrid, padding_mode='border', align_corners=True, mode='bilinear')
    return c.squeeze(-1).squeeze(-1).transpose(1, 2).squeeze(0)


def _lin(x, prm, name):
    return F.linear(x, prm[name + '.weight'], prm[name + '.bias'])


def mlp_forward(p, grids, prm, pre, name, bound, color=False, concat=False):
    """decoder.py:190-219 (MLP.forward, fourier embedding, skips=[2])."""
    c = sample_grid_feature(p, grids['grid_' + name], bound, 'grid_' + name)
    if concat:  # decoder.py:196-202: middle feature concatenated without grad
        with torch.no_grad():
            c_mid = sample_grid_feature(p, grids['grid_middle'], bound, 'grid_middle')
        c = torch.cat([c, c_mid], dim=1)
    pf = _in32(p)
    emb = torch.sin(pf @ prm[pre + 'embedder._B'])  # decoder.py:26-30
    h = emb
    for i in range(5):
        h = F.relu(_lin(h, prm, f'{pre}pts_linears.{i}'))
        h = h + _lin(c, prm, f'{pre}fc_c.{i}')
        if i == 2:
            h = torch.cat([emb, h], -1)
    out = _lin(h, prm, pre + 'output_linear')
    return out if color else out.squeeze(-1)


def mlp_no_xyz_forward(p, grids, prm, pre, bound):
    """decoder.py:285-297 (coarse decoder)."""
    c = sample_grid_feature(p, grids['grid_coarse'], bound, 'grid_coarse')
    h = c
    for i in range(5):
        h = F.relu(_lin(h, prm, f'{pre}pts_linears.{i}'))
        if i == 2:
            h = torch.cat([c, h], -1)
    return _lin(h, prm, pre + 'output_linear').squeeze(-1)


def nice_forward(p, grids, prm, dec_bounds, stage):
    """decoder.py:336-370 — raw [P,4]; color-decoder channel 3 is overwritten."""
    P = p.shape[0]
    if stage == 'coarse':
        occ = mlp_no_xyz_forward(p, grids, prm, 'coarse_decoder.', dec_bounds['coarse'])
        raw = torch.zeros(P, 4, dtype=FLOAT)
        raw[..., -1] = occ
        return raw
    if stage == 'middle':
        occ = mlp_forward(p, grids, prm, 'middle_decoder.', 'middle', dec_bounds['middle'])
        raw = torch.zeros(P, 4, dtype=FLOAT)
        raw[..., -1] = occ
        return raw
    fine_occ = mlp_forward(p, grids, prm, 'fine_decoder.', 'fine', dec_bounds['fine'], concat=True)
    if stage == 'fine':
        raw = torch.zeros(P, 4, dtype=FLOAT)
    else:
        raw = mlp_forward(p, grids, prm, 'color_decoder.', 'color', dec_bounds['color'], color=True)
    mid_occ = mlp_forward(p, grids, prm, 'middle_decoder.', 'middle', dec_bounds['middle'])
    raw[..., -1] = fine_occ + mid_occ
    return raw


def eval_points(p, grids, prm, bound, dec_bounds, stage):
    """Renderer.py:36-93 — strict in-bound mask against the renderer bound,
    out-of-bound points get raw[:,3] = 100."""
    mask = ((p[:, 0] < bound[0][1]) & (p[:, 0] > bound[0][0]) &
            (p[:, 1] < bound[1][1]) & (p[:, 1] > bound[1][0]) &
            (p[:, 2] < bound[2][1]) & (p[:, 2] > bound[2][0]))
    ret = nice_forward(p, grids, prm, dec_bounds, stage)
    ret[~mask, 3] = 100
    return ret


def sample_depths(rays_o, rays_d, bound, gt_depth, n_strat, n_surf, depth_max=None, lindisp=False,
                  t_rand=None):
    """Renderer.py:116-224 — z_vals [N, S] float64 (stratified + surface, sorted).
    ``depth_max`` (sharding tests only) replaces the batch-global max(gt_depth).
    ``lindisp`` (Renderer.py:208-209) and ``t_rand`` (perturb > 0, :211-219: the
    [N, n_strat] float32 draws the reference takes from torch.rand)."""
    N = rays_o.shape[0]
    if gt_depth is None:
        n_surf = 0
        near = 0.01
    else:
        gt_depth = gt_depth.reshape(-1, 1)
        near = gt_depth.repeat(1, n_strat) * 0.01
    with torch.no_grad():
        o = rays_o.clone().detach().unsqueeze(-1)
        d = rays_d.clone().detach().unsqueeze(-1)
        t = (bound.unsqueeze(0) - o) / d
        far_bb, _ = torch.min(torch.max(t, dim=2)[0], dim=1)
        far_bb = far_bb.unsqueeze(-1) + 0.01
    gmax = None
    if gt_depth is not None:
        gmax = torch.max(gt_depth) if depth_max is None else depth_max.reshape(())
    far = torch.clamp(far_bb, 0, gmax * 1.2) if gt_depth is not None else far_bb
    if n_surf > 0:
        pos = gt_depth > 0
        ts = torch.linspace(0., 1., steps=n_surf).double()
        zs = torch.zeros(N, n_surf).double()
        g = gt_depth[pos].unsqueeze(-1).repeat(1, n_surf)
        zs[pos.squeeze(-1), :] = 0.95 * g * (1. - ts) + 1.05 * g * ts
        zs[~pos.squeeze(-1), :] = 0.001 * (1. - ts) + gmax * ts
    tv = torch.linspace(0., 1., steps=n_strat)
    if not lindisp:
        z = near * (1. - tv) + far * tv
    else:
        z = 1. / (1. / near * (1. - tv) + 1. / far * (tv))
    if t_rand is not None:
        mids = .5 * (z[..., 1:] + z[..., :-1])
        upper = torch.cat([mids, z[..., -1:]], -1)
        lower = torch.cat([z[..., :1], mids], -1)
        z = lower + (upper - lower) * t_rand
    if n_surf > 0:
        z, _ = torch.sort(torch.cat([z, zs.double()], -1), -1)
    return z


def composite(raw, z_vals):
    """common.py:215-256 with occupancy=True: alpha = sigmoid(10 occ), exclusive
    cumprod of (1-alpha+1e-10); rgb, depth (f64) and depth variance (f64)."""
    rgb = raw[..., :-1]
    alpha = torch.sigmoid(10 * raw[..., -1])
    ones = torch.ones((alpha.shape[0], 1), dtype=FLOAT)
    weights = alpha.to(FLOAT) * torch.cumprod(torch.cat([ones, (1. - alpha + 1e-10).to(FLOAT)], -1), -1)[:, :-1]
    rgb_map = torch.sum(weights[..., None] * rgb, -2)
    depth_map = torch.sum(weights * z_vals, -1)
    tmp = z_vals - depth_map.unsqueeze(-1)
    depth_var = torch.sum(weights * tmp * tmp, dim=1)
    return depth_map, depth_var, rgb_map, weights


def render_batch_ray(grids, prm, dec_bounds, bound, rays_d, rays_o, stage, gt_depth=None,
                     n_strat=32, n_surf=16, depth_max=None, n_importance=0, lindisp=False, t_rand=None):
    """Renderer.py:95-262 (occupancy on; lindisp, and perturb through its draws t_rand;
    hierarchical sampling with sample_pdf, :239-259, when n_importance > 0).
    Returns (depth f64 [N], uncertainty f64 [N], color f32 [N,3])."""
    if stage == 'coarse':
        gt_depth = None
    z = sample_depths(rays_o, rays_d, bound, gt_depth, n_strat, n_surf, depth_max, lindisp, t_rand)
    S = z.shape[1]
    pts = rays_o[..., None, :] + rays_d[..., None, :] * z[..., :, None]
    raw = eval_points(pts.reshape(-1, 3), grids, prm, bound, dec_bounds, stage)
    raw = raw.reshape(rays_o.shape[0], S, -1)
    depth, var, color, weights = composite(raw, z)
    if n_importance > 0:
        from oracle.pdf_oracle import sample_pdf
        z_mid = .5 * (z[..., 1:] + z[..., :-1])
        z_samples = sample_pdf(z_mid, weights[..., 1:-1], n_importance, det=True).detach()
        z, _ = torch.sort(torch.cat([z, z_samples], -1), -1)
        pts = rays_o[..., None, :] + rays_d[..., None, :] * z[..., :, None]
        raw = eval_points(pts.reshape(-1, 3), grids, prm, bound, dec_bounds, stage)
        raw = raw.reshape(rays_o.shape[0], S + n_importance, -1)
        depth, var, color, _ = composite(raw, z)
    return depth, var, color


def get_rays(H, W, fx, fy, cx, cy, c2w):
    """common.py:259-277 get_rays: one ray per pixel, pixel centres at integer
    coordinates, camera looking down -z; c2w [4,4] float32."""
    i, j = torch.meshgrid(torch.linspace(0, W - 1, W), torch.linspace(0, H - 1, H), indexing="ij")
    i, j = i.t(), j.t()
    dirs = torch.stack([(i - cx) / fx, -(j - cy) / fy, -torch.ones_like(i)], -1).reshape(H, W, 1, 3)
    rays_d = torch.sum(dirs * c2w[:3, :3], -1)
    rays_o = c2w[:3, -1].expand(rays_d.shape)
    return rays_o, rays_d


def render_img(grids, prm, dec_bounds, bound, H, W, fx, fy, cx, cy, c2w, stage, gt_depth=None,
               ray_batch_size=100000):
    """Renderer.py:264-340 render_img: get_rays, then render_batch_ray over chunks of
    ray_batch_size rays (each chunk with its own max(gt_depth), as the reference's
    per-call batch max), depth/uncertainty as float64 [H,W], color [H,W,3].
    (The reference reshapes gt_depth unconditionally, so gt_depth=None raises there;
    here it renders without depth.)"""
    with torch.no_grad():
        rays_o, rays_d = get_rays(H, W, fx, fy, cx, cy, c2w)
        rays_o, rays_d = rays_o.reshape(-1, 3), rays_d.reshape(-1, 3)
        gt = gt_depth.reshape(-1) if gt_depth is not None else None
        dl, ul, cl = [], [], []
        for s in range(0, rays_d.shape[0], ray_batch_size):
            e = s + ray_batch_size
            d, u, c = render_batch_ray(grids, prm, dec_bounds, bound, rays_d[s:e], rays_o[s:e], stage,
                                       None if gt is None else gt[s:e])
            dl.append(d.double()); ul.append(u.double()); cl.append(c)
        return torch.cat(dl).reshape(H, W), torch.cat(ul).reshape(H, W), torch.cat(cl).reshape(H, W, 3)


def mapper_loss(depth, color, gt_depth, gt_color=None, w_color=0.2, color_term=False):
    """Mapper.optimize_map's rendering loss (Mapper.py:603-612, nice=True, occupancy on):
    L1 depth over gt > 0 (float64) plus, in the 'color' stage, w_color times the
    unmasked float32 L1 colour sum.  Parity of the loss itself is UNPINNED (the
    reference's loss lives inside Mapper.optimize_map; no fixture holds it) -- its
    inputs, the render outputs, are pinned by tests/golden."""
    m = gt_depth > 0
    loss = torch.abs(gt_depth[m] - depth[m]).sum()
    if color_term:
        loss = loss + w_color * torch.abs(gt_color - color).sum()
    return loss


def tracker_loss(depth, var, color, gt_depth, gt_color=None, w_color=0.5, color_term=True,
                 handle_dynamic=True):
    """Tracker.optimize_cam_in_batch's loss (Tracker.py:117-131): depth residual scaled
    by the detached render uncertainty, rays with gt > 0 (and, with handle_dynamic,
    residual < 10 x its lower median -- torch.median) only; the optional colour term
    uses the same mask.  Parity unpinned, as mapper_loss."""
    var = var.detach()
    scaled = torch.abs(gt_depth - depth) / torch.sqrt(var + 1e-10)
    if handle_dynamic:
        mask = (scaled < 10 * scaled.median()) & (gt_depth > 0)
    else:
        mask = gt_depth > 0
    loss = scaled[mask].sum()
    if color_term:
        loss = loss + w_color * torch.abs(gt_color - color)[mask].sum()
    return loss


def points_for_rays(rays_o, rays_d, bound, gt_depth, stage, n_strat=32, n_surf=16):
    """The float64 sample points render_batch_ray evaluates (Renderer.py:227-231)."""
    if stage == 'coarse':
        gt_depth = None
    z = sample_depths(rays_o, rays_d, bound, gt_depth, n_strat, n_surf)
    return z, (rays_o[..., None, :].double() + rays_d[..., None, :].double() * z[..., :, None])


def params_from_module(nice) -> dict:
    """name -> tensor view of a NICE module's parameters (reference names)."""
    return dict(nice.named_parameters())
