"""Host-side logic that needs no GPU: decoder module parity with the reference's
parameter names / seeded init, bound snapping and grid shapes."""
import numpy as np
import torch

from conftest import load_scene
from nicecore import decoder as D
from nicecore import scene as S

ADJUSTED = {"coarse_decoder.output_linear.bias", "middle_decoder.output_linear.bias",
            "fine_decoder.output_linear.bias"}  # biased by make_golden.py


def test_nice_param_names_and_seeded_init_match_reference():
    _, _, _, params = load_scene()
    m = D.build_default_nice(seed=0)
    named = dict(m.named_parameters())
    assert list(named) == list(params)  # same registration order as the reference
    for k, v in named.items():
        assert v.shape == params[k].shape, k
        if k not in ADJUSTED:
            assert torch.equal(v.detach(), params[k]), k
    assert sum(p.numel() for p in m.parameters()) == 58956


def test_bound_snapping_matches_reference_fixture():
    bound, cbound, grids, _ = load_scene()
    sc = S.make_scene("tiny")
    assert torch.equal(sc.bound, bound)
    assert torch.equal(S.decoder_bounds(sc.bound)["coarse"], cbound)
    for k, g in grids.items():
        assert list(g.shape[2:]) == sc.shapes[k], k


def test_replica_room0_bound_and_shapes():
    # room0 grids coarse [7,8,11] middle [21,28,37] fine/color [43,56,74];
    # x-max snaps to 8.94000015258789 through the float32 product.
    sc = S.make_scene("replica_room0")
    assert abs(float(sc.bound[0, 1]) - 8.94000015258789) < 1e-12
    assert sc.shapes["grid_coarse"] == [7, 8, 11]
    assert sc.shapes["grid_middle"] == [21, 28, 37]
    assert sc.shapes["grid_fine"] == [43, 56, 74]
    assert sc.shapes["grid_color"] == [43, 56, 74]
    assert S.make_scene("scannet_scene0000").shapes["grid_fine"] == [47, 85, 81]
    assert S.make_scene("apartment").shapes["grid_middle"] == [40, 26, 53]


def test_synth_rays_pass_bbox_filter():
    sc = S.make_scene("replica_room0")
    ro, rd, dep, col = S.synth_rays(sc, 500, seed=3)
    t = S.ray_exit_t(sc.bound, ro, rd)
    assert bool((t >= dep.double()).all())
    assert (dep == 0).float().mean() > 0.03


def _model_with_bounds():
    m = D.build_default_nice(seed=0)
    b = S.make_scene("tiny").bound
    m.bound = b
    for n in ("middle", "fine", "color"):
        getattr(m, n + "_decoder").bound = b
    m.coarse_decoder.bound = b * 2
    return m


def test_plan_cache_reuse_and_invalidation():
    """The per-decoders binding is reused while the parameters are the same objects
    and storage, and rebuilt when a parameter object, its storage or a bound changes."""
    from nicecore import _lib as L
    from nicecore.render_fn import make_plan, decoder_params
    m = _model_with_bounds()
    p1 = make_plan("color", m)
    assert make_plan("color", m) is p1
    assert make_plan("middle", m) is not p1
    # ABI order == decoder_params == fast path
    for k in p1.decs:
        assert all(a is b for a, b in zip(p1.params[k], decoder_params(p1.modules[k], k)))
    img = p1.decoder_image(torch.device("cpu"))
    w0 = m.fine_decoder.pts_linears[0].weight
    assert img[L.DEC_FINE].lin_w[0] == w0.data_ptr()
    # .data swap keeps the object but moves the storage -> image refreshed
    w0.data = w0.data.clone()
    img2 = p1.decoder_image(torch.device("cpu"))
    assert make_plan("color", m) is p1
    assert img2[L.DEC_FINE].lin_w[0] == w0.data_ptr()
    # a replaced Parameter object -> new plan
    m.fine_decoder.pts_linears[0].weight = torch.nn.Parameter(w0.detach().clone())
    p2 = make_plan("color", m)
    assert p2 is not p1
    assert p2.params[L.DEC_FINE][11] is m.fine_decoder.pts_linears[0].weight
    # a new bound object -> new plan
    m.fine_decoder.bound = m.fine_decoder.bound.clone()
    assert make_plan("color", m) is not p2


def test_render_template_fields():
    from nicecore import _lib as L
    from nicecore.render_fn import make_plan
    m = _model_with_bounds()
    plan = make_plan("color", m)
    b = m.bound
    t = plan.render_template(torch.device("cpu"), 32, 16, b)
    assert t.abi_version == L.NC_ABI_VERSION and t.stage == 3 and (t.n_strat, t.n_surf) == (32, 16)
    ts, tsurf = S.linspace_tables(32, 16)
    assert [t.t_strat[k] for k in range(32)] == ts.tolist()
    assert [t.t_surf[k] for k in range(16)] == tsurf.tolist()
    assert t.bound[0][1] == float(b[0, 1])
    assert t.dec[L.DEC_COLOR].out_w == m.color_decoder.output_linear.weight.data_ptr()
    assert plan.render_template(torch.device("cpu"), 32, 16, b) is t


def test_graph_live_accumulator_scan():
    """nicecore.graph._live_accumulators finds the gradient accumulators of an autograd
    graph held only by a container (the round-4 capture_end crash pattern),
    and forgets them once the graph is dropped."""
    import torch
    from nicecore.graph import _live_accumulators
    a = torch.zeros(3, requires_grad=True)
    b = torch.ones(2, requires_grad=True)
    held = {"loss": (a * 2).sum() + (b * b).sum()}
    leaves = list(_live_accumulators().values())
    assert any(v is a for v in leaves) and any(v is b for v in leaves)
    held.clear()
    assert not any(v is a or v is b for v in _live_accumulators().values())
