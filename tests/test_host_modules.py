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
