"""NC_SAVE_POINT_JACOBIAN: the forward keeps d features / d (ix, iy, iz) of every decoder
lookup and the backward's coordinate gradient contracts it with d features, instead of
re-reading the 8 grid corners (the reference's grid_sampler_3d_backward gix/giy/giz,
decoder.py:186).  Both paths are reassociations of the same sums: ray / point gradients
agree to 1e-5 of max-abs; every other gradient is bit-identical (they do not depend on
the coordinate gradient).  The golden-vector parity tests run with the Jacobian on
(the default)."""
import pytest
import torch

from parity_common import rel_err
from test_gpu_determinism import _render_grads
from test_gpu_parity import _room0_case


@pytest.mark.gpu
@pytest.mark.parametrize("stage", ["color", "middle", "coarse"])
def test_jacobian_matches_corner_rereads(stage, monkeypatch):
    from nicecore import render_fn
    sc, grids, params, ro, rd, dep = _room0_case(384, stage, seed=61)
    monkeypatch.setattr(render_fn, "_SAVE_JAC", True)
    a = _render_grads(sc, grids, params, ro, rd, dep, stage, True)
    monkeypatch.setattr(render_fn, "_SAVE_JAC", False)
    b = _render_grads(sc, grids, params, ro, rd, dep, stage, True)
    assert a.keys() == b.keys()
    for k in a:
        if k in ("grad/rays_o", "grad/rays_d"):
            assert rel_err(a[k], b[k]) <= 1e-5, (k, rel_err(a[k], b[k]))
        else:
            assert torch.equal(a[k], b[k]), k


@pytest.mark.gpu
def test_jacobian_eval_points(monkeypatch):
    """NICE.forward on caller points (nc_points_*): d p with and without the Jacobian."""
    from nicecore import render_fn
    from nicecore.ops import eval_points
    from parity_common import build_model
    sc, grids, params, ro, rd, dep = _room0_case(8, "color", seed=67)
    model = build_model(params, sc.bound, sc.bound * 2, "cuda")
    g = {k: v.cuda() for k, v in grids.items()}
    gen = torch.Generator().manual_seed(2)
    lo, hi = sc.bound[:, 0], sc.bound[:, 1]
    p0 = (lo + (hi - lo) * torch.rand(3000, 3, generator=gen, dtype=torch.float64)).float().cuda()
    up = torch.randn(3000, 4, generator=gen).cuda()
    out = []
    for jac in (True, False):
        monkeypatch.setattr(render_fn, "_SAVE_JAC", jac)
        p = p0.clone().requires_grad_(True)
        (eval_points(model, p, g, "color") * up).sum().backward()
        out.append(p.grad.detach().clone())
    assert rel_err(out[0], out[1]) <= 1e-5, rel_err(out[0], out[1])
