"""lindisp and perturb > 0 (src/utils/Renderer.py:208-219) against golden vectors the
reference renderer itself produced (tests/golden/make_golden_strat.py, its perturbation
draws stored as ``t_rand``): the CPU oracle (pins it) and the HIP path (ABI v9
``nc_render_args.lindisp`` / ``.t_rand``), both through the drop-in Renderer and with the
caller-given draws."""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, load_scene
from oracle import nice_oracle as O

META = json.load(open(os.path.join(GOLDEN, "strat_meta.json")))
CASES = [c["name"] for c in META["cases"]]
OUT_TOL, GRAD_TOL = 2e-5, 2e-4


def _case(name):
    c = next(x for x in META["cases"] if x["name"] == name)
    with np.load(os.path.join(GOLDEN, f"case_{name}.npz")) as z:
        rec = {k: torch.from_numpy(z[k]) for k in z.files}
    return c, rec


@pytest.mark.parametrize("name", CASES)
def test_oracle_matches_reference(name):
    c, rec = _case(name)
    bound, cbound, grids, params = load_scene()
    ro = rec["rays_o"].clone().requires_grad_(True)
    rd = rec["rays_d"].clone().requires_grad_(True)
    g = {k: v.clone().requires_grad_(True) for k, v in grids.items()}
    prm = {k: v.clone().requires_grad_(True) for k, v in params.items()}
    dec_b = {"coarse": cbound, "middle": bound, "fine": bound, "color": bound}
    gt = rec["gt_depth"] if c["with_depth"] else None
    d, v, col = O.render_batch_ray(g, prm, dec_b, bound, rd, ro, c["stage"], gt, META["n_samples"],
                                   META["n_surface"], lindisp=c["lindisp"], t_rand=rec.get("t_rand"))
    torch.autograd.backward([d, v, col], [rec["g_depth"], rec["g_var"], rec["g_color"]])
    torch.testing.assert_close(d.detach(), rec["depth"], rtol=1e-12, atol=1e-13)
    torch.testing.assert_close(v.detach(), rec["var"], rtol=1e-12, atol=1e-13)
    torch.testing.assert_close(col.detach(), rec["color"], rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(ro.grad, rec["grad/rays_o"], rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(rd.grad, rec["grad/rays_d"], rtol=1e-5, atol=1e-6)
    for k, t in list(g.items()) + [("param/" + n, p) for n, p in prm.items()]:
        key = "grad/" + k
        if key in rec:
            torch.testing.assert_close(t.grad, rec[key], rtol=1e-5, atol=1e-6)


def test_renderer_accepts_the_options():
    """The drop-in Renderer no longer refuses lindisp / perturb for NICE decoders (the
    iMAP* path still does: configs/imap.yaml has both off)."""
    import types
    from nicecore.renderer import Renderer
    cfg = {"rendering": {"N_samples": 32, "N_surface": 16, "N_importance": 0, "lindisp": True, "perturb": 1.0},
           "scale": 1, "occupancy": True}
    slam = types.SimpleNamespace(nice=True, bound=torch.zeros(3, 2), H=4, W=4, fx=1., fy=1., cx=1., cy=1.)
    Renderer(cfg, None, slam)._check_supported()
    cfg["occupancy"] = False
    slam.nice = False
    with pytest.raises(NotImplementedError):
        Renderer(cfg, None, slam)._check_supported()


def _rel(a, b):
    a, b = a.detach().double().cpu().reshape(-1), b.double().reshape(-1)
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
@pytest.mark.parametrize("channels_last", [False, True])
def test_hip_matches_reference(name, channels_last):
    import types
    from nicecore.renderer import Renderer
    from parity_common import build_model
    c, rec = _case(name)
    bound, cbound, grids, params = load_scene()
    model = build_model(params, bound, cbound, "cuda")
    g = {}
    for k, v in grids.items():
        t = v.cuda()
        if channels_last:
            t = t.contiguous(memory_format=torch.channels_last_3d)
        g[k] = t.requires_grad_(True)
    cfg = {"rendering": {"N_samples": META["n_samples"], "N_surface": META["n_surface"], "N_importance": 0,
                         "lindisp": c["lindisp"], "perturb": c["perturb"]}, "scale": 1, "occupancy": True}
    slam = types.SimpleNamespace(nice=True, bound=bound, H=48, W=64, fx=40., fy=40., cx=31.5, cy=23.5)
    r = Renderer(cfg, None, slam)
    ro = rec["rays_o"].cuda().requires_grad_(True)
    rd = rec["rays_d"].cuda().requires_grad_(True)
    gt = rec["gt_depth"].cuda() if c["with_depth"] else None
    tr = rec["t_rand"].cuda() if "t_rand" in rec else None
    d, v, col = r.render_batch_ray(g, model, rd, ro, "cuda", c["stage"], gt, t_rand=tr)
    torch.autograd.backward([d, v, col], [rec["g_depth"].cuda(), rec["g_var"].cuda(), rec["g_color"].cuda()])
    errs = {"depth": _rel(d, rec["depth"]), "var": _rel(v, rec["var"]), "color": _rel(col, rec["color"]),
            "grad/rays_o": _rel(ro.grad, rec["grad/rays_o"]), "grad/rays_d": _rel(rd.grad, rec["grad/rays_d"])}
    for k, t in g.items():
        if "grad/" + k in rec:
            errs["grad/" + k] = _rel(t.grad, rec["grad/" + k])
    for n, p in model.named_parameters():
        if "grad/param/" + n in rec:
            errs["grad/param/" + n] = _rel(p.grad, rec["grad/param/" + n])
    bad = {k: e for k, e in errs.items() if not e <= (GRAD_TOL if k.startswith("grad/") else OUT_TOL)}
    assert not bad, bad


@pytest.mark.gpu
def test_hip_perturb_draws_from_cpu_generator():
    """Without t_rand the Renderer draws torch.rand([N, N_samples]) on the CPU's default
    generator, as the reference: re-seeding reproduces the render."""
    import types
    from nicecore.renderer import Renderer
    from parity_common import build_model
    c, rec = _case("strat_perturb_color_depth")
    bound, cbound, grids, params = load_scene()
    model = build_model(params, bound, cbound, "cuda")
    g = {k: v.cuda() for k, v in grids.items()}
    cfg = {"rendering": {"N_samples": 32, "N_surface": 16, "N_importance": 0, "lindisp": False, "perturb": 1.0},
           "scale": 1, "occupancy": True}
    slam = types.SimpleNamespace(nice=True, bound=bound, H=48, W=64, fx=40., fy=40., cx=31.5, cy=23.5)
    r = Renderer(cfg, None, slam)
    ro, rd, gt = rec["rays_o"].cuda(), rec["rays_d"].cuda(), rec["gt_depth"].cuda()
    with torch.no_grad():
        torch.manual_seed(7)
        a = r.render_batch_ray(g, model, rd, ro, "cuda", "color", gt)
        torch.manual_seed(7)
        t = torch.rand(ro.shape[0], 32)
        b = r.render_batch_ray(g, model, rd, ro, "cuda", "color", gt, t_rand=t.cuda())
    for x, y in zip(a, b):
        assert torch.equal(x, y)
