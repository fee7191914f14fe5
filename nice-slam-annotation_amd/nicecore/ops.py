"""Functional entry points of the render core (HIP only, no fallback)."""
from __future__ import annotations

import torch

from . import _lib as L
from .render_fn import NiceEvalFn, NiceRenderFn, make_plan


def _grid_args(c):
    return [c.get(k) if c is not None else None for k in L.GRID_KEYS]


def eval_points(decoders, p, c_grid, stage='middle'):
    """NICE.forward(p, c_grid, stage) (src/conv_onet/models/decoder.py:336-370):
    raw [P,4] float32 for points p ([P,3] or [1,P,3]); differentiable w.r.t. p,
    the grids and the decoder parameters."""
    plan = make_plan(stage, decoders)
    spec = {"plan": plan}
    return NiceEvalFn.apply(spec, p, *_grid_args(c_grid), *plan.flat_params())


def render_rays(decoders, c, rays_o, rays_d, bound, stage, gt_depth=None, n_strat=32,
                n_surf=16, depth_max=None):
    """Renderer.render_batch_ray core (src/utils/Renderer.py:95-262) with
    N_importance = 0, lindisp = False, perturb = 0, occupancy = True.
    Returns (depth float64 [N], uncertainty float64 [N], color float32 [N,3]).

    ``depth_max``: optional device scalar replacing the batch-global max(gt_depth)
    (Renderer.py:157, :194) -- pass the all-reduced max when a batch is sharded."""
    if stage == 'coarse':
        gt_depth = None
    ns = n_surf if gt_depth is not None else 0
    if n_strat + ns > L.NC_MAX_SAMPLES or ns > L.NC_MAX_SURF:
        raise L.NiceCoreError("nicecore supports N_samples + N_surface <= 64 (N_surface <= 32)")
    plan = make_plan(stage, decoders)
    spec = {"plan": plan, "n_strat": n_strat, "n_surf": ns, "bound": bound, "depth_max": depth_max}
    return NiceRenderFn.apply(spec, rays_o, rays_d, gt_depth, *_grid_args(c), *plan.flat_params())
