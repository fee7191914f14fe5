"""Weight images prebuilt by the forward (csrc/nc_wimage.h).

k_ray_setup / k_points_prep build k_mlp_fwd's split-f16 image and, for a forward that
saves for the backward, k_mlp_dx's f32 image: the backward reads the weights the forward
used, as the reference's nn.Linear saves its weight for backward
(/root/reference/src/conv_onet/models/decoder.py:209-216).  A decoder parameter changed
in place between the forward and its backward is therefore an autograd error, as in the
reference; a fresh forward after the change sees the new weights."""
import pytest
import torch

from conftest import load_case, load_scene
from parity_common import build_model, make_renderer


def _setup():
    bound, cbound, grids, params = load_scene()
    rec = load_case("color_depth")
    model = build_model(params, bound, cbound, "cuda")
    g = {k: v.cuda().contiguous(memory_format=torch.channels_last_3d) for k, v in grids.items()}
    return bound, rec, model, g


@pytest.mark.gpu
def test_render_inplace_weight_change_raises():
    bound, rec, model, g = _setup()
    ro, rd = rec["rays_o"].cuda().requires_grad_(True), rec["rays_d"].cuda().requires_grad_(True)
    d, v, c = make_renderer(bound).render_batch_ray(g, model, rd, ro, "cuda", "color", rec["gt_depth"].cuda())
    w = model.fine_decoder.fc_c[1].weight
    with torch.no_grad():
        w.mul_(2.0)
    with pytest.raises(RuntimeError, match="modified by an inplace operation"):
        (d.sum() + c.sum()).backward()


@pytest.mark.gpu
def test_points_inplace_weight_change_raises():
    _, rec, model, g = _setup()
    raw = model(rec["pts"].cuda(), g, "color")
    with torch.no_grad():
        model.color_decoder.pts_linears[2].bias.add_(0.5)
    with pytest.raises(RuntimeError, match="modified by an inplace operation"):
        raw.sum().backward()


@pytest.mark.gpu
def test_images_rebuilt_per_forward():
    """A weight change between two forwards reaches the second one (the images are
    rebuilt by every forward, not cached)."""
    _, rec, model, g = _setup()
    pts = rec["pts"].cuda()
    with torch.no_grad():
        a = model(pts, g, "color").clone()
        model.color_decoder.output_linear.bias.add_(1.0)
        b = model(pts, g, "color")
    assert torch.allclose(b[:, :3], a[:, :3] + 1.0, atol=1e-5)
    assert torch.equal(b[:, 3], a[:, 3])


def _run_all(model, g, rec, bound):
    ro, rd = rec["rays_o"].cuda().requires_grad_(True), rec["rays_d"].cuda().requires_grad_(True)
    for p in model.parameters():
        p.grad = None
    d, v, c = make_renderer(bound).render_batch_ray(g, model, rd, ro, "cuda", "color", rec["gt_depth"].cuda())
    (d.sum() + v.sum() + c.sum()).backward()
    out = {"depth": d.detach(), "var": v.detach(), "color": c.detach(), "g_ro": ro.grad, "g_rd": rd.grad}
    out.update({"p/" + n: p.grad.clone() for n, p in model.named_parameters() if p.grad is not None})
    with torch.no_grad():
        out["raw"] = model(rec["pts"].cuda(), g, "color")
    torch.cuda.synchronize()
    return out


@pytest.mark.gpu
def test_images_cover_their_workspace(monkeypatch):
    """The builders write every 16-B chunk of both images (no zero fill): a workspace whose
    bytes are all 0xFF (NaN as floats) before the call gives bit-identical outputs and
    decoder / ray gradients."""
    bound, rec, model, g = _setup()
    clean = _run_all(model, g, rec, bound)
    real_empty = torch.empty

    def poisoned(*a, **kw):
        t = real_empty(*a, **kw)
        if kw.get("dtype") is torch.uint8 and t.is_cuda:
            t.fill_(255)
        return t

    monkeypatch.setattr(torch, "empty", poisoned)
    dirty = _run_all(model, g, rec, bound)
    monkeypatch.setattr(torch, "empty", real_empty)
    for k, t in clean.items():
        assert torch.equal(t, dirty[k]), k
