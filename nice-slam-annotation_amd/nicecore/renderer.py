"""Drop-in ``Renderer`` (src/utils/Renderer.py:5-341) on the MI355X render core.

Same constructor, attributes and method signatures as the reference, so
src/Tracker.py / src/Mapper.py / src/utils/Visualizer.py call it unchanged:

  render_batch_ray(c, decoders, rays_d, rays_o, device, stage, gt_depth=None)
      -> (depth f64 [N], uncertainty f64 [N], color f32 [N,3])      Renderer.py:95
  eval_points(p, decoders, c=None, stage='color', device='cuda:0')
      -> raw [P,4]                                                    Renderer.py:36
  render_img(c, decoders, c2w, device, stage, gt_depth=None)
      -> (depth [H,W], uncertainty [H,W], color [H,W,3])              Renderer.py:264

plus ``render_batch_loss`` (extension): render_batch_ray with the Mapper's / Tracker's
loss expression (Mapper.py:603-612, Tracker.py:117-131) computed in the same launches.

Implemented: the NICE decoders with occupancy = True (configs/nice_slam.yaml:5,121-126),
lindisp and perturb (Renderer.py:208-219; perturb's draws are torch.rand on the CPU's
default generator as in the reference, or the caller's ``t_rand``) and any N_importance
(hierarchical sampling, Renderer.py:239-259); iMAP* (slam.nice = False: one scene MLP,
occupancy = False volume density, N_surface = 0, lindisp = False, perturb = 0,
configs/imap.yaml) through nicecore.imap, plus its ``regulation`` (Renderer.py:343-409);
anything else raises instead of silently falling back.
"""
from __future__ import annotations

import torch

from . import _lib as L
from . import imap as _imap
from .ops import eval_points as _eval_points
from .ops import render_rays, render_rays_loss


class Renderer(object):
    def __init__(self, cfg, args, slam, points_batch_size=500000, ray_batch_size=100000):
        self.ray_batch_size = ray_batch_size
        self.points_batch_size = points_batch_size
        r = cfg['rendering']
        self.lindisp = r['lindisp']
        self.perturb = r['perturb']
        self.N_samples = r['N_samples']
        self.N_surface = r['N_surface']
        self.N_importance = r['N_importance']
        # extension: how the decoder parameters get their .grad ("autograd" | "direct",
        # render_fn.param_inputs); absent from the reference configs = the default
        self.param_grads = r.get('param_grads')
        self.scale = cfg['scale']
        self.occupancy = cfg['occupancy']
        self.nice = slam.nice
        self.bound = slam.bound
        self.H, self.W, self.fx, self.fy, self.cx, self.cy = (
            slam.H, slam.W, slam.fx, slam.fy, slam.cx, slam.cy)

    def _check_supported(self):
        if not self.nice and (self.lindisp or self.perturb > 0.):
            raise NotImplementedError("nicecore's iMAP* path implements lindisp=False, perturb=0 (configs/imap.yaml)")
        if self.nice != self.occupancy:
            raise NotImplementedError(
                "nicecore renders NICE decoders with occupancy=True (configs/nice_slam.yaml) and the "
                "iMAP* MLP with volume density, occupancy=False (configs/imap.yaml)")
        if not self.nice and self.N_surface != 0:
            raise NotImplementedError("iMAP* renders with N_surface = 0 (configs/imap.yaml:108)")

    def eval_points(self, p, decoders, c=None, stage='color', device='cuda:0'):
        """Renderer.py:36-93: NICE.forward plus the strict in-bound mask; points outside
        the renderer bound get raw[:, 3] = 100."""
        self._check_supported()
        # Chunks write into one output allocated from the first chunk's dtype and device
        # (what the decoders return, as the reference's cat) and the bound mask is applied
        # once over all points (elementwise identical to the per-chunk mask).
        b = self.bound
        out = None
        s = 0
        for pi in torch.split(p, self.points_batch_size):
            r = _eval_points(decoders, pi, c, stage) if self.nice else _imap.eval_points(decoders, pi)
            if out is None:
                out = torch.empty(p.shape[0], 4, dtype=r.dtype, device=r.device)
            out[s:s + pi.shape[0]] = r
            s += pi.shape[0]
        if out is None:  # no chunk at all
            out = torch.empty(0, 4, dtype=torch.float32, device=p.device)
        m = ((p[:, 0] < b[0][1]) & (p[:, 0] > b[0][0]) & (p[:, 1] < b[1][1]) &
             (p[:, 1] > b[1][0]) & (p[:, 2] < b[2][1]) & (p[:, 2] > b[2][0]))
        out[:, 3].masked_fill_(~m, 100.0)
        return out

    def render_batch_ray(self, c, decoders, rays_d, rays_o, device, stage, gt_depth=None,
                         depth_max=None, sparse_grads=None, t_rand=None, ray_mask=None):
        """Renderer.py:95-262.  Extensions: ``depth_max`` overrides the batch-global
        max(gt_depth) with a precomputed (e.g. all-reduced) device scalar;
        ``sparse_grads`` (nicecore.sparse.SparseGridGrads) takes the covered grids'
        gradients as touched-voxel rows (grids too large for a dense gradient);
        ``t_rand`` ([N, N_samples]) gives perturb's draws instead of torch.rand;
        ``ray_mask`` ([N] bool, e.g. sampling.sample_frames' ``inside``) drops the rays the
        callers' bbox pre-filter rejects without compacting the batch (ops.render_rays)."""
        self._check_supported()
        if gt_depth is not None:
            gt_depth = gt_depth.reshape(-1)
        if not self.nice:  # iMAP*: the scene MLP + volume density (nicecore.imap)
            if ray_mask is not None:
                raise NotImplementedError("ray_mask is the NICE callers' bbox pre-filter (Tracker.py:99, Mapper.py:580)")
            return _imap.render_rays(decoders, rays_o, rays_d, self.bound, gt_depth, self.N_samples,
                                     self.N_importance, depth_max)
        return render_rays(decoders, c, rays_o, rays_d, self.bound, stage, gt_depth,
                           self.N_samples, self.N_surface, depth_max, sparse_grads=sparse_grads,
                           n_importance=self.N_importance, perturb=self.perturb, lindisp=self.lindisp,
                           t_rand=t_rand, param_grads=self.param_grads, ray_mask=ray_mask)

    def render_batch_loss(self, c, decoders, rays_d, rays_o, device, stage, gt_depth, gt_color=None,
                          loss='mapper', w_color_loss=0.2, color_term=False, handle_dynamic=False,
                          render_gt_depth='target', depth_max=None, sparse_grads=None,
                          defer_param_grads=None, t_rand=None, ray_mask=None):
        """render_batch_ray + the rendering loss (ops.render_rays_loss): returns
        (depth, uncertainty, color, loss).  Mapper.optimize_map:
        ``loss='mapper', color_term=(not nice) or stage == 'color',
        render_gt_depth=None if coarse_mapper else 'target'``; Tracker.optimize_cam_in_batch:
        ``loss='tracker', color_term=use_color_in_tracking, handle_dynamic=handle_dynamic``."""
        self._check_supported()
        if not self.nice:
            raise NotImplementedError("render_batch_loss fuses the NICE losses; iMAP* callers use render_batch_ray")
        return render_rays_loss(decoders, c, rays_o, rays_d, self.bound, stage, gt_depth.reshape(-1),
                                loss, gt_color, w_color_loss, color_term, handle_dynamic,
                                render_gt_depth, self.N_samples, self.N_surface, depth_max,
                                sparse_grads=sparse_grads, n_importance=self.N_importance,
                                perturb=self.perturb, defer_param_grads=defer_param_grads,
                                lindisp=self.lindisp, t_rand=t_rand, param_grads=self.param_grads,
                                ray_mask=ray_mask)

    def regulation(self, c, decoders, rays_d, rays_o, gt_depth, device, stage='color', t_rand=None):
        """Renderer.py:343-409 (iMAP* only): densities of N_samples points per ray in
        [0, 0.85 gt_depth], stratified with random offsets (perturb = 1); the decoder runs on
        the HIP core (eval_points).  ``t_rand`` ([N, N_samples], default torch.rand) makes the
        draw reproducible."""
        S = self.N_samples
        # near = 0: z = 0 * (1 - t) + far * t == far * t exactly
        z = (gt_depth.reshape(-1, 1) * 0.85) * torch.linspace(0., 1., steps=S).to(device)
        mid = .5 * (z[:, 1:] + z[:, :-1])
        lo, hi = torch.cat([z[:, :1], mid], 1), torch.cat([mid, z[:, -1:]], 1)
        if t_rand is None:
            t_rand = torch.rand(z.shape).to(device)
        z = lo + (hi - lo) * t_rand
        pts = (rays_o[:, None, :] + rays_d[:, None, :] * z[:, :, None]).reshape(-1, 3)
        return self.eval_points(pts, decoders, c, stage, device)[:, 3]

    def render_img(self, c, decoders, c2w, device, stage, gt_depth=None):
        """Renderer.py:264-340: chunked full-image render, no grad."""
        with torch.no_grad():
            H, W = self.H, self.W
            i, j = torch.meshgrid(torch.linspace(0, W - 1, W), torch.linspace(0, H - 1, H),
                                  indexing='ij')
            i, j = i.t(), j.t()
            dirs = torch.stack([(i - self.cx) / self.fx, -(j - self.cy) / self.fy,
                                -torch.ones_like(i)], -1).to(device)
            c2w = torch.as_tensor(c2w, device=device)
            rays_d = torch.sum(dirs[..., None, :] * c2w[:3, :3], -1).reshape(-1, 3).float()
            rays_o = c2w[:3, -1].expand(rays_d.shape).reshape(-1, 3).float()
            gt = gt_depth.reshape(-1) if gt_depth is not None else None
            dl, ul, cl = [], [], []
            for s in range(0, rays_d.shape[0], self.ray_batch_size):
                d, u, col = self.render_batch_ray(
                    c, decoders, rays_d[s:s + self.ray_batch_size], rays_o[s:s + self.ray_batch_size],
                    device, stage, gt_depth=None if gt is None else gt[s:s + self.ray_batch_size])
                dl.append(d.double()); ul.append(u.double()); cl.append(col)
            return (torch.cat(dl).reshape(H, W), torch.cat(ul).reshape(H, W),
                    torch.cat(cl).reshape(H, W, 3))
