"""Shared setup for GPU parity runs: build the drop-in Renderer + NICE on a HIP
device from the golden scene, render a golden case, back-propagate the stored
upstream gradients and collect every output / input gradient."""
from __future__ import annotations

import types

import numpy as np
import torch

from conftest import load_case, load_meta, load_scene
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
    c = next(c for c in load_meta()["cases"] if c["name"] == name)
    return c["stage"], c["with_depth"]


def run_case(name, device="cuda", channels_last=False, want=("rays", "grids", "params")):
    bound, cbound, grids, params = load_scene()
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
