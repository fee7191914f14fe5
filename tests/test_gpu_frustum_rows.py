"""The Mapper's per-iteration frustum feature selection on the device (nicecore.frustum
MaskedGrid, nc_grid_rows): val[mask].clone() (src/Mapper.py:393-404), val[mask] = val_grad
with its autograd (:491-500), the write-back after the optimiser step (:633-642).  Every
result is a plain copy, so each one is held bit-exact to ATen's boolean-index /
index_put on the same GPU tensors, for channels-last and NCDHW grids, and end to end
through a deterministic render of the scattered grid."""
import pytest
import torch

from parity_common import build_model, make_renderer


def _grid(shape, channels_last, seed):
    g = torch.randn(1, 32, *shape, generator=torch.Generator().manual_seed(seed)).cuda()
    return g.contiguous(memory_format=torch.channels_last_3d) if channels_last else g


def _mask(shape, seed, frac=0.3):
    return (torch.rand(shape, generator=torch.Generator().manual_seed(seed)) < frac).cuda()


@pytest.mark.gpu
@pytest.mark.parametrize("channels_last", [True, False])
@pytest.mark.parametrize("shape", [(21, 28, 37), (3, 5, 7), (1, 1, 1)])
def test_select_scatter_writeback_equal_aten(channels_last, shape):
    from nicecore.frustum import MaskedGrid
    val = _grid(shape, channels_last, 1)
    m3 = _mask(shape, 2)
    m3.view(-1)[0] = True  # at least one voxel
    m5 = m3[None, None].repeat(1, 32, 1, 1, 1)  # Mapper.py:394-395
    sel = MaskedGrid(m5)
    assert sel.n == int(m3.sum())
    vg = sel.select(val)
    assert torch.equal(vg, val[m5].clone())
    new = torch.randn(vg.shape, generator=torch.Generator().manual_seed(3)).cuda()
    ours = val.clone(memory_format=torch.preserve_format)
    ref = val.clone(memory_format=torch.preserve_format)
    sel.scatter_(ours, new)
    ref[m5] = new
    assert torch.equal(ours, ref)
    assert ours.stride() == val.stride()
    # write-back (no autograd)
    wb = sel.write_back_(val.clone(memory_format=torch.preserve_format), new * 2)
    ref2 = val.clone()
    ref2[m5] = new * 2
    assert torch.equal(wb, ref2)


@pytest.mark.gpu
@pytest.mark.parametrize("channels_last", [True, False])
def test_scatter_autograd_equals_index_put(channels_last):
    """d val_grad = grad[mask] and d val = grad with the masked voxels zeroed, as
    IndexPutBackward gives them."""
    from nicecore.frustum import MaskedGrid
    shape = (9, 11, 13)
    base = _grid(shape, channels_last, 4)
    m3 = _mask(shape, 5)
    m5 = m3[None, None].repeat(1, 32, 1, 1, 1)
    sel = MaskedGrid(m3)
    w = torch.randn(base.shape, generator=torch.Generator().manual_seed(6)).cuda()
    outs = []
    for ours in (True, False):
        b = base.clone().requires_grad_(True)
        vg = b.detach()[m5].clone().requires_grad_(True)
        val = b * 1.0  # non-leaf, as the Mapper's val after .to(device)
        if ours:
            sel.scatter_(val, vg)
        else:
            val[m5] = vg
        (val * w).sum().backward()
        outs.append((vg.grad, b.grad))
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])


@pytest.mark.gpu
def test_mapper_frustum_iteration_through_render(monkeypatch):
    """One Mapper iteration in the frustum mode (Mapper.py:491-500, :598-612): the
    masked voxels scattered into the grids, render_batch_ray + loss, backward into
    val_grad; ordered (NC_DETERMINISTIC) grid scatter so both paths see the same dense
    gradient: val_grad.grad equal to the index_put path's bit for bit."""
    from nicecore import scene as S
    from nicecore.frustum import FrustumSelector, MaskedGrid
    from test_gpu_parity import _room0_case
    monkeypatch.setenv("NC_DETERMINISTIC", "1")
    sc, grids, params, ro, rd, dep = _room0_case(200, "color", seed=61)
    model = build_model(params, sc.bound, sc.bound * 2, "cuda")
    r = make_renderer(sc.bound, H=sc.H, W=sc.W)
    poses = []
    S.synth_rays(sc, 1, seed=62, poses_out=poses)
    R, t = poses[0]
    c2w = torch.eye(4)
    c2w[:3, :3], c2w[:3, 3] = R, t
    depth = torch.full((sc.H, sc.W), 6.0)
    fs = FrustumSelector(sc.bound, sc.H, sc.W, sc.fx, sc.fy, sc.cx, sc.cy, "cuda")
    keys = ("grid_middle", "grid_fine", "grid_color")
    res = []
    for ours in (True, False):
        c = {k: v.cuda().contiguous(memory_format=torch.channels_last_3d) for k, v in grids.items()}
        vgs = {}
        for k in keys:
            m3 = fs.grid_mask(c2w, k, c[k].shape[2:], depth)
            m5 = m3[None, None].repeat(1, 32, 1, 1, 1)
            if ours:
                sel = MaskedGrid(m3)
                vgs[k] = sel.select(c[k]).requires_grad_(True)
                sel.scatter_(c[k], vgs[k])
            else:
                vgs[k] = c[k][m5].clone().requires_grad_(True)
                c[k][m5] = vgs[k]
        d, u, col = r.render_batch_ray(c, model, rd.cuda(), ro.cuda(), "cuda", "color", dep.cuda())
        loss = (dep.cuda().double() - d).abs().sum() + 0.2 * col.abs().sum()
        loss.backward()
        res.append({k: vgs[k].grad.clone() for k in keys})
        for p in model.parameters():
            p.grad = None
    for k in keys:
        assert float(res[0][k].abs().max()) > 0, k
        assert torch.equal(res[0][k], res[1][k]), k
