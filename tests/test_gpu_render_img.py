"""Renderer.render_img (Renderer.py:264-340; SURVEY.md §8f rank 1, forward-only reuse of
the render core for the Visualizer) vs the oracle's restatement (oracle/nice_oracle.py
render_img: common.py:259-277 get_rays + chunked render_batch_ray) on the tiny golden
scene, a whole 48x64 image.  Chunking matters: each chunk of ray_batch_size rays uses
its own max(gt_depth) in the reference, so a chunked render differs from a one-shot
render and both are checked.  Tolerance: the render parity bar (2e-5 of max-abs)."""
import pytest
import torch

from conftest import load_scene
from parity_common import build_model, make_renderer, rel_err
from oracle import nice_oracle as O


def _camera():
    th = 0.3
    c2w = torch.eye(4)
    c2w[:3, :3] = torch.tensor([[1.0, 0.0, 0.0],
                                [0.0, torch.cos(torch.tensor(th)), -torch.sin(torch.tensor(th))],
                                [0.0, torch.sin(torch.tensor(th)), torch.cos(torch.tensor(th))]])
    c2w[:3, 3] = torch.tensor([0.1, -0.05, 0.45])
    return c2w


@pytest.mark.gpu
@pytest.mark.parametrize("stage,with_depth,chunk", [("color", True, 100000), ("color", True, 1000),
                                                    ("middle", True, 777), ("fine", False, 100000),
                                                    ("coarse", False, 2048)])
def test_render_img_matches_oracle(stage, with_depth, chunk):
    bound, cbound, grids, params = load_scene()
    r = make_renderer(bound)
    r.ray_batch_size = chunk
    H, W = r.H, r.W
    model = build_model(params, bound, cbound, "cuda")
    g = {k: v.cuda() for k, v in grids.items()}
    c2w = _camera()
    gen = torch.Generator().manual_seed(4)
    gt = torch.rand(H, W, generator=gen) * 0.7 + 0.1
    gt[torch.rand(H, W, generator=gen) < 0.1] = 0.0
    gt_in = gt.cuda() if with_depth else None
    d, u, c = r.render_img(g, model, c2w.cuda(), "cuda", stage, gt_depth=gt_in)
    assert d.shape == (H, W) and u.shape == (H, W) and c.shape == (H, W, 3)
    assert d.dtype == torch.float64 and u.dtype == torch.float64 and c.dtype == torch.float32
    dec_bounds = {"coarse": cbound, "middle": bound, "fine": bound, "color": bound}
    rd_, ru, rc = O.render_img(grids, params, dec_bounds, bound, H, W, r.fx, r.fy, r.cx, r.cy, c2w, stage,
                               gt if with_depth else None, ray_batch_size=chunk)
    assert rel_err(d.cpu(), rd_) <= 2e-5
    assert rel_err(u.cpu(), ru) <= 2e-5
    if stage == "color":
        assert rel_err(c.cpu(), rc) <= 2e-5


@pytest.mark.gpu
def test_render_img_chunks_use_their_own_depth_max():
    """The chunked image differs from a one-shot render where a chunk's max(gt_depth)
    differs from the image's (the reference's per-call batch max, Renderer.py:157)."""
    bound, cbound, grids, params = load_scene()
    r = make_renderer(bound)
    model = build_model(params, bound, cbound, "cuda")
    g = {k: v.cuda() for k, v in grids.items()}
    gt = torch.full((r.H, r.W), 0.3)
    gt[-1, -1] = 0.9  # only the last chunk sees the large depth
    r.ray_batch_size = 1000
    d1, _, _ = r.render_img(g, model, _camera().cuda(), "cuda", "color", gt_depth=gt.cuda())
    r.ray_batch_size = 100000
    d2, _, _ = r.render_img(g, model, _camera().cuda(), "cuda", "color", gt_depth=gt.cuda())
    assert not torch.equal(d1[:10], d2[:10])
