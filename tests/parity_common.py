"""Shared setup for GPU parity runs: build the drop-in Renderer + NICE on a HIP
device from the golden scene, render a golden case, back-propagate the stored
upstream gradients and collect every output / input gradient."""
from __future__ import annotations

import types

import numpy as np
import torch

from conftest import load_case, load_initstd_meta, load_meta, load_scene
from nicecore import decoder as D
from nicecore import scene as S
from nicecore.renderer import Renderer

CFG = {"rendering": dict(S.DEFAULT_RENDERING), "scale": 1, "occupancy": True}


def build_model(params, bound, cbound, device):
    m = D.build_default_nice(seed=0)
    m.load_state_dict(params)
    m = m.to(device)
    b = bound.to(device)
    m.bound = b
    for n in ("middle", "fine", "color"):
        getattr(m, n + "_decoder").bound = b
    m.coarse_decoder.bound = cbound.to(device)
    return m


def make_renderer(bound, H=48, W=64):
    slam = types.SimpleNamespace(nice=True, bound=bound, H=H, W=W, fx=40.0, fy=40.0, cx=31.5, cy=23.5)
    return Renderer(CFG, None, slam)


def case_stage(name):
    cases = load_meta()["cases"] + load_initstd_meta()["cases"]
    c = next(c for c in cases if c["name"] == name)
    return c["stage"], c["with_depth"]


def scene_of(name):
    """Golden scene a case was rendered on (make_golden.py / make_golden_initstd.py)."""
    return "initstd" if name.startswith("initstd_") else "tiny"


def run_case(name, device="cuda", channels_last=False, want=("rays", "grids", "params")):
    bound, cbound, grids, params = load_scene(scene_of(name))
    rec = load_case(name)
    stage, with_depth = case_stage(name)
    model = build_model(params, bound, cbound, device)
    for p in model.parameters():
        p.requires_grad_("params" in want)
    g = {}
    for k, v in grids.items():
        t = v.to(device)
        if channels_last:
            t = t.contiguous(memory_format=torch.channels_last_3d)
        g[k] = t.requires_grad_("grids" in want)
    ro = rec["rays_o"].to(device).requires_grad_("rays" in want)
    rd = rec["rays_d"].to(device).requires_grad_("rays" in want)
    gt = rec["gt_depth"].to(device) if with_depth else None
    r = make_renderer(bound)
    depth, var, color = r.render_batch_ray(g, model, rd, ro, device, stage, gt)
    torch.autograd.backward([depth, var, color],
                            [rec["g_depth"].to(device), rec["g_var"].to(device), rec["g_color"].to(device)])
    got = {"depth": depth.detach(), "var": var.detach(), "color": color.detach()}
    if "rays" in want:
        got["grad/rays_o"] = ro.grad
        got["grad/rays_d"] = rd.grad
    if "grids" in want:
        for k, v in g.items():
            if v.grad is not None:
                got["grad/" + k] = v.grad
    if "params" in want:
        for n, p in model.named_parameters():
            if p.grad is not None:
                got["grad/param/" + n] = p.grad
    return rec, {k: v.detach().cpu() for k, v in got.items()}


def rel_err(got, ref):
    """max |got - ref| / max(|ref|_max, tiny) — scale-aware error of a whole tensor."""
    got = got.double().reshape(-1)
    ref = ref.double().reshape(-1)
    scale = float(ref.abs().max()) if ref.numel() else 0.0
    return float((got - ref).abs().max()) / max(scale, 1e-30) if ref.numel() else 0.0


def compare(rec, got):
    out = {}
    for k, v in got.items():
        if k in rec:
            out[k] = rel_err(v, rec[k])
        else:
            out[k] = float(v.abs().max())  # reference has no gradient here -> must be ~0
    return out


def oracle_render_grads(grids, params, dec_b, bound, ro, rd, stage, gt, upstream, f64=False, depth_max=None):
    """CPU oracle render + backward; with f64=True everything runs in float64
    (ground truth).  ``depth_max``: the batch-global max(gt_depth) of a sharded batch.
    Returns {name: tensor} like run_case."""
    from oracle import nice_oracle as O
    cast = (lambda t: t.double()) if f64 else (lambda t: t)
    ro_c = cast(ro.clone()).requires_grad_(True)
    rd_c = cast(rd.clone()).requires_grad_(True)
    g_c = {k: cast(v.clone()).requires_grad_(True) for k, v in grids.items()}
    prm_c = {k: cast(v.clone()).requires_grad_(True) for k, v in params.items()}
    gt_c = cast(gt) if gt is not None else None
    ctx = O.float64_mode() if f64 else _null()
    with ctx:
        dm = None if depth_max is None else cast(depth_max.reshape(()).clone())
        d, v, c = O.render_batch_ray(g_c, prm_c, dec_b, bound, rd_c, ro_c, stage, gt_c, depth_max=dm)
        gd, gv, gc = upstream
        torch.autograd.backward([d, v, c], [gd, gv, cast(gc)])
    out = {"depth": d.detach(), "var": v.detach(), "color": c.detach(),
           "grad/rays_o": ro_c.grad, "grad/rays_d": rd_c.grad}
    for k, t in g_c.items():
        if t.grad is not None and float(t.grad.abs().max()) > 0:
            out["grad/" + k] = t.grad
    for k, t in prm_c.items():
        if t.grad is not None and float(t.grad.abs().max()) > 0:
            out["grad/param/" + k] = t.grad
    return out


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def score_vs_truth(got, ref32, ref64, out_floor=2e-5, grad_floor=2e-4):
    """{name: (err_hip, err_ref32, allowed)} where err = scale-aware error vs float64."""
    res = {}
    for k, t64 in ref64.items():
        if k not in got:
            res[k] = (float("inf"), 0.0, 0.0)
            continue
        e_hip = rel_err(got[k], t64)
        e_ref = rel_err(ref32[k], t64) if k in ref32 else 0.0
        floor = grad_floor if k.startswith("grad/") else out_floor
        res[k] = (e_hip, e_ref, max(4.0 * e_ref, floor))
    return res
