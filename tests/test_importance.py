"""Hierarchical sampling inside render_batch_ray (N_importance > 0, Renderer.py:239-259):
a forward-only first pass, sample_pdf over its weights (without the first and last
sample) at the mid-points of its depths, then the differentiable render over the sorted
union of both sample sets.  Golden vectors from the reference's own Renderer with
rendering.N_importance = 8 / 12 (tests/golden/make_golden_importance.py).

The importance depths are a step function of the first pass's float32 weights,
amplified by 1 / (cdf[above] - cdf[below]) (sample_pdf's t), so float32 rounding that
differs by an ulp -- another CPU's vectorised sums, or the MFMA decoders -- moves them
measurably.  CPU: the oracle against the goldens; in the build container that made
them it is exact to 1e-12 (outputs), on another host's CPU it agrees to 2e-6; bar 1e-5
outputs / 1e-3 gradients, of each tensor's max-abs.  GPU: the drop-in Renderer (two nc_render_forward passes
around nc_sample_pdf) against the goldens: outputs 2e-5 of each tensor's max-abs as the
N_importance = 0 parity, or 4x the largest departure of three unit-permuted float32 oracles
(8.6e-6 on imp_middle_nodepth's var: another float32 summation order moves an importance
depth as far), gradients 1e-3 (2.6e-4 measured: sums over points that moved)."""
import pytest
import torch

from conftest import load_case, load_meta, load_scene
from oracle import nice_oracle as O

CASES = ["imp_color_depth", "imp_middle_nodepth"]


def _case(name):
    rec = load_case(name)
    stage = ["coarse", "middle", "fine", "color"][int(rec["stage"])]
    return rec, stage, bool(rec["with_depth"]), int(rec["n_importance"])


@pytest.mark.parametrize("name", CASES)
def test_oracle_importance_matches_reference(name):
    meta = load_meta()
    rec, stage, with_depth, nimp = _case(name)
    bound, cbound, grids, params = load_scene()
    ro = rec["rays_o"].clone().requires_grad_(True)
    rd = rec["rays_d"].clone().requires_grad_(True)
    g = {k: v.clone().requires_grad_(True) for k, v in grids.items()}
    prm = {k: v.clone().requires_grad_(True) for k, v in params.items()}
    dec_bounds = {"coarse": cbound, "middle": bound, "fine": bound, "color": bound}
    depth, var, color = O.render_batch_ray(g, prm, dec_bounds, bound, rd, ro, stage,
                                           rec["gt_depth"] if with_depth else None,
                                           meta["n_samples"], meta["n_surface"], n_importance=nimp)
    torch.autograd.backward([depth, var, color], [rec["g_depth"], rec["g_var"], rec["g_color"]])
    from parity_common import rel_err
    outs = {"depth": (depth, rec["depth"]), "var": (var, rec["var"]), "color": (color, rec["color"])}
    for k, (a, b) in outs.items():
        assert rel_err(a.detach(), b) <= 1e-5, (k, rel_err(a.detach(), b))
    grads = {"rays_o": (ro.grad, rec["grad/rays_o"]), "rays_d": (rd.grad, rec["grad/rays_d"])}
    grads.update({k: (v.grad, rec["grad/" + k]) for k, v in g.items() if "grad/" + k in rec})
    grads.update({k: (v.grad, rec["grad/param/" + k]) for k, v in prm.items() if "grad/param/" + k in rec})
    bad = {k: rel_err(a, b) for k, (a, b) in grads.items() if rel_err(a, b) > 1e-3}
    assert not bad, bad


def _permuted_spread(name, seeds=(1, 2, 3)):
    """max over unit-permuted float32 oracles of their departure from the reference's vectors."""
    from parity_common import permuted_problem, rel_err
    meta = load_meta()
    rec, stage, with_depth, nimp = _case(name)
    bound, cbound, grids, params = load_scene()
    dec_b = {"coarse": cbound, "middle": bound, "fine": bound, "color": bound}
    out = {"depth": 0.0, "var": 0.0, "color": 0.0}
    for seed in seeds:
        g2, p2, _ = permuted_problem(grids, params, seed)
        with torch.no_grad():
            d, v, c = O.render_batch_ray(g2, p2, dec_b, bound, rec["rays_d"], rec["rays_o"], stage,
                                         rec["gt_depth"] if with_depth else None, meta["n_samples"],
                                         meta["n_surface"], n_importance=nimp)
        for k, t in (("depth", d), ("var", v), ("color", c)):
            out[k] = max(out[k], rel_err(t, rec[k]))
    return out


def test_permuted_spread_is_small():
    """The spread the GPU bar allows stays at float32 level (< 1e-4 of max-abs)."""
    for name in CASES:
        sp = _permuted_spread(name)
        assert max(sp.values()) < 1e-4, (name, sp)


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_hip_importance_matches_reference(name):
    import types
    from nicecore import scene as S
    from nicecore.renderer import Renderer
    from parity_common import build_model, rel_err
    rec, stage, with_depth, nimp = _case(name)
    bound, cbound, grids, params = load_scene()
    model = build_model(params, bound, cbound, "cuda")
    g = {k: v.cuda().contiguous(memory_format=torch.channels_last_3d).requires_grad_(True)
         for k, v in grids.items()}
    ro = rec["rays_o"].cuda().requires_grad_(True)
    rd = rec["rays_d"].cuda().requires_grad_(True)
    cfg = {"rendering": dict(S.DEFAULT_RENDERING, N_importance=nimp), "scale": 1, "occupancy": True}
    slam = types.SimpleNamespace(nice=True, bound=bound, H=48, W=64, fx=40.0, fy=40.0, cx=31.5, cy=23.5)
    r = Renderer(cfg, None, slam)
    gt = rec["gt_depth"].cuda() if with_depth else None
    depth, var, color = r.render_batch_ray(g, model, rd, ro, "cuda", stage, gt)
    torch.autograd.backward([depth, var, color],
                            [rec["g_depth"].cuda(), rec["g_var"].cuda(), rec["g_color"].cuda()])
    errs = {"depth": rel_err(depth.detach().cpu(), rec["depth"]),
            "var": rel_err(var.detach().cpu(), rec["var"]),
            "color": rel_err(color.detach().cpu(), rec["color"])}
    # the bar: 2e-5 of max-abs, or 4x the largest departure of three other float32
    # implementations (the unit-permuted oracles: the same function, every dot product summed
    # in another order) -- the importance depths jump with the first pass's last ulps, so an
    # independent float32 implementation lands as far off on the rays whose pdf bins tie
    spread = _permuted_spread(name)
    bar = {k: max(2e-5, 4.0 * spread[k]) for k in errs}
    print(f"\n[{name}] HIP vs reference {errs}; permuted float32 spread {spread}")
    assert all(errs[k] <= bar[k] for k in errs), (errs, bar)
    gerr = {"rays_o": rel_err(ro.grad.cpu(), rec["grad/rays_o"]), "rays_d": rel_err(rd.grad.cpu(), rec["grad/rays_d"])}
    for k, v in g.items():
        if "grad/" + k in rec:
            gerr[k] = rel_err(v.grad.cpu(), rec["grad/" + k])
    for n, p in model.named_parameters():
        if "grad/param/" + n in rec:
            gerr[n] = rel_err(p.grad.cpu(), rec["grad/param/" + n])
    assert max(gerr.values()) <= 1e-3, {k: v for k, v in gerr.items() if v > 1e-3}
