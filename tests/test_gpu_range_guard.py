"""Split-f16 range guard of k_mlp_fwd (csrc/nc_device.h RANGE_LIMIT, nc_mlp.hip
k_mlp_fwd_exact).

The forward decoder GEMMs split each f32 operand into f16 hi + scaled f16 lo; that is
exact to f32 level only for |x| < 2^15.  Trained grids and decoders are not bounded, so
every split operand's magnitude is tracked, and a job that saw one at or above 2^15 (or
an infinite one) is recomputed whole on the exact-f32 MFMA.  These tests drive the
operands far past 65504 -- grid features (the fc_c and MLP_no_xyz inputs), decoder
weights, and hidden activations -- and hold the result to the reference's fp32 addmm
semantics (the oracle, decoder.py:209-216) at the usual tolerances, through
NICE.forward (nc_points_*) and render_batch_ray (nc_render_*, with gradients)."""
import pytest
import torch

from conftest import load_case, load_scene
from parity_common import build_model, make_renderer, rel_err

OUT_TOL = 2e-5
GRAD_TOL = 2e-4


def _scaled(what, scale):
    bound, cbound, grids, params = load_scene()
    grids = {k: v.clone() for k, v in grids.items()}
    params = {k: v.clone() for k, v in params.items()}
    if what == "grid":  # features ~ 1e5 x the fixture's
        for k in grids:
            grids[k] = grids[k] / grids[k].abs().max() * scale
    elif what == "weight":  # one fc_c matrix per decoder ~ scale
        for dec in ("middle", "fine", "color"):
            w = params[f"{dec}_decoder.fc_c.1.weight"]
            params[f"{dec}_decoder.fc_c.1.weight"] = w / w.abs().max() * scale
        w = params["coarse_decoder.pts_linears.1.weight"]
        params["coarse_decoder.pts_linears.1.weight"] = w / w.abs().max() * scale
    elif what == "bias":  # hidden activations ~ scale (block 1 biases), split as block 2's input
        for dec in ("coarse", "middle", "fine", "color"):
            params[f"{dec}_decoder.pts_linears.1.bias"] = params[f"{dec}_decoder.pts_linears.1.bias"] + scale
    return bound, cbound, grids, params


@pytest.mark.gpu
@pytest.mark.parametrize("what,scale", [("grid", 2.0e5), ("weight", 7.0e4), ("bias", 1.0e5), ("grid", 3.0e4)])
@pytest.mark.parametrize("stage", ["color", "middle", "coarse"])
def test_points_forward_past_f16_range(what, scale, stage):
    from oracle import nice_oracle as O
    bound, cbound, grids, params = _scaled(what, scale)
    pts = load_case("color_depth")["pts"]
    dec_b = {"coarse": cbound, "middle": bound, "fine": bound, "color": bound}
    with torch.no_grad():
        ref = O.nice_forward(pts.clone(), grids, params, dec_b, stage)
    assert float(ref.abs().max()) > 1e3  # the operands really are large
    model = build_model(params, bound, cbound, "cuda")
    g = {k: v.cuda().contiguous(memory_format=torch.channels_last_3d) for k, v in grids.items()}
    with torch.no_grad():
        raw = model(pts.cuda(), g, stage).cpu()
    assert bool(torch.isfinite(raw).all())
    assert rel_err(raw[:, 3], ref[:, 3]) <= OUT_TOL, rel_err(raw[:, 3], ref[:, 3])
    if stage == "color":
        assert rel_err(raw[:, :3], ref[:, :3]) <= OUT_TOL


@pytest.mark.gpu
@pytest.mark.parametrize("what,scale", [("grid", 2.0e5), ("bias", 1.0e5), ("weight", 7.0e4)])
def test_render_past_f16_range_with_gradients(what, scale):
    """render_batch_ray + backward: the backward reads the activation records the exact
    recompute wrote (relu masks, h_L), so its gradients are the f32 path's."""
    from parity_common import oracle_render_grads
    bound, cbound, grids, params = _scaled(what, scale)
    rec = load_case("color_depth")
    dec_b = {"coarse": cbound, "middle": bound, "fine": bound, "color": bound}
    up = (rec["g_depth"], rec["g_var"], rec["g_color"])
    ref = oracle_render_grads(grids, params, dec_b, bound, rec["rays_o"], rec["rays_d"], "color", rec["gt_depth"], up)
    model = build_model(params, bound, cbound, "cuda")
    g = {k: v.cuda().contiguous(memory_format=torch.channels_last_3d).requires_grad_(True) for k, v in grids.items()}
    ro, rd = rec["rays_o"].cuda().requires_grad_(True), rec["rays_d"].cuda().requires_grad_(True)
    d, v, c = make_renderer(bound).render_batch_ray(g, model, rd, ro, "cuda", "color", rec["gt_depth"].cuda())
    torch.autograd.backward([d, v, c], [t.cuda() for t in up])
    got = {"depth": d, "var": v, "color": c, "grad/rays_o": ro.grad, "grad/rays_d": rd.grad}
    got.update({"grad/" + k: t.grad for k, t in g.items() if t.grad is not None})
    got.update({"grad/param/" + n: p.grad for n, p in model.named_parameters() if p.grad is not None})
    for k, r in ref.items():
        tol = GRAD_TOL if k.startswith("grad/") else OUT_TOL
        e = rel_err(got[k].detach().cpu(), r)
        assert e <= tol, (k, e)
