"""ORACLE — TEST INFRASTRUCTURE ONLY.  Never imported by the product path.

CPU restatement of the iMAP* render path (configs/imap.yaml: ``slam.nice = False``,
``occupancy: False``, N_surface = 0) over torch CPU ops with the reference's op
order and dtypes:

  * the scene MLP of ``get_model(cfg, nice=False)`` (src/conv_onet/config.py:28-32):
    MLP.forward with c_dim = 0, hidden 256, 4 blocks, no skip (decoder.py:190-219);
  * ``raw2outputs_nerf_color(..., occupancy=False)`` (src/common.py:215-256): volume
    density alpha = 1 - exp(-relu(raw) * dists), dists scaled by ||rays_d||;
  * ``Renderer.render_batch_ray`` (Renderer.py:95-262) with those two, reusing the
    NICE oracle's sampling (nice_oracle.sample_depths) and sample_pdf (pdf_oracle).

Parity status: PINNED — tests/test_oracle_golden.py::test_imap_* checks it against
tests/golden/imap_*.npz, captured from the reference itself by
tests/golden/make_golden_imap.py.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from oracle import nice_oracle as NO


def imap_forward(p, prm, masks=None):
    """decoder.py:190-219 with c_dim = 0 (no grid feature, no skip): raw [P,4].
    ``masks`` (tests only): per hidden layer a [P,256] bool tensor imposed in place of
    relu's own branch, h = z * mask -- the same piecewise-linear function evaluated on
    given ReLU branches (a float64 truth on the branches an fp32 evaluation took)."""
    emb = torch.sin(p.to(NO.FLOAT) @ prm['embedder._B'])  # decoder.py:26-30
    h = emb
    for i in range(4):
        z = F.linear(h, prm[f'pts_linears.{i}.weight'], prm[f'pts_linears.{i}.bias'])
        h = F.relu(z) if masks is None else z * masks[i].to(z.dtype)
    return F.linear(h, prm['output_linear.weight'], prm['output_linear.bias'])


def imap_relu_masks(p, prm):
    """The ReLU branches (z > 0) of imap_forward's four hidden layers, [P,256] bool each, in
    the current compute dtype (tests: how many (point, unit) branches an fp32 evaluation
    takes differently from float64)."""
    with torch.no_grad():
        h = torch.sin(p.to(NO.FLOAT) @ prm['embedder._B'])
        out = []
        for i in range(4):
            z = F.linear(h, prm[f'pts_linears.{i}.weight'], prm[f'pts_linears.{i}.bias'])
            out.append(z > 0)
            h = F.relu(z)
    return out


def eval_points(p, prm, bound):
    """Renderer.py:36-93 with nice = False: decoders(pi, c_grid=None), strict in-bound
    mask, raw[~mask, 3] = 100."""
    mask = ((p[:, 0] < bound[0][1]) & (p[:, 0] > bound[0][0]) &
            (p[:, 1] < bound[1][1]) & (p[:, 1] > bound[1][0]) &
            (p[:, 2] < bound[2][1]) & (p[:, 2] > bound[2][0]))
    ret = imap_forward(p, prm)
    ret[~mask, 3] = 100
    return ret


def composite_density(raw, z_vals, rays_d):
    """common.py:232-256 with occupancy = False."""
    dists = (z_vals[..., 1:] - z_vals[..., :-1]).float()
    dists = torch.cat([dists, torch.full_like(dists[..., :1], 1e10)], -1)
    dists = dists * torch.norm(rays_d[..., None, :], dim=-1)
    rgb = raw[..., :-1]
    alpha = 1. - torch.exp(-F.relu(raw[..., -1]) * dists)
    ones = torch.ones((alpha.shape[0], 1), dtype=NO.FLOAT)
    weights = alpha.to(NO.FLOAT) * torch.cumprod(torch.cat([ones, (1. - alpha + 1e-10).to(NO.FLOAT)], -1), -1)[:, :-1]
    rgb_map = torch.sum(weights[..., None] * rgb, -2)
    depth_map = torch.sum(weights * z_vals, -1)
    tmp = z_vals - depth_map.unsqueeze(-1)
    depth_var = torch.sum(weights * tmp * tmp, dim=1)
    return depth_map, depth_var, rgb_map, weights


def render_batch_ray(prm, bound, rays_d, rays_o, gt_depth=None, n_strat=32, n_importance=0, depth_max=None):
    """Renderer.py:95-262 for iMAP* (N_surface = 0, lindisp / perturb off).
    Returns (depth f64 [N], uncertainty f64 [N], color f32 [N,3])."""
    z = NO.sample_depths(rays_o, rays_d, bound, gt_depth, n_strat, 0, depth_max)
    S = z.shape[1]
    N = rays_o.shape[0]
    pts = rays_o[..., None, :] + rays_d[..., None, :] * z[..., :, None]
    raw = eval_points(pts.reshape(-1, 3), prm, bound).reshape(N, S, -1)
    depth, var, color, weights = composite_density(raw, z, rays_d)
    if n_importance > 0:
        from oracle.pdf_oracle import sample_pdf
        z_mid = .5 * (z[..., 1:] + z[..., :-1])
        z_samples = sample_pdf(z_mid, weights[..., 1:-1], n_importance, det=True).detach()
        z, _ = torch.sort(torch.cat([z, z_samples], -1), -1)
        pts = rays_o[..., None, :] + rays_d[..., None, :] * z[..., :, None]
        raw = eval_points(pts.reshape(-1, 3), prm, bound).reshape(N, S + n_importance, -1)
        depth, var, color, _ = composite_density(raw, z, rays_d)
    return depth, var, color


def params_from_module(mlp) -> dict:
    return {k: v.detach().clone() for k, v in mlp.named_parameters()}
