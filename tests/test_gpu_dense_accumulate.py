"""A C caller that runs nc_render_backward twice into the same dense gradient buffer
(no zero fill between) gets the sum of both (ABI: grid gradients are accumulated into
``nc_grid.grad``; nicecore.h) in both scatter modes: float atomics, and NC_DETERMINISTIC,
whose per-voxel run sums are read-add-written (nc_det.hip det_add / k_det_runs).  The
decoder weight gradients are written, not accumulated, so they come out unchanged."""
import ctypes

import pytest
import torch

from parity_common import rel_err
from test_gpu_defer import _setup


@pytest.mark.gpu
@pytest.mark.parametrize("deterministic", [False, True])
def test_second_backward_adds_into_grid_gradients(deterministic, monkeypatch):
    from nicecore import _lib as L
    if deterministic:
        monkeypatch.setenv("NC_DETERMINISTIC", "1")
    sc, g, model, ro, rd, gt, gtc, r = _setup()
    d, u, c, loss = r.render_batch_loss(g, model, rd, ro, "cuda", "color", gt, gtc, loss="mapper", color_term=True)
    loss.backward()
    torch.cuda.synchronize()
    first = {k: t.grad.detach().clone() for k, t in g.items() if t.grad is not None}
    pfirst = {n: p.grad.detach().clone() for n, p in model.named_parameters() if p.grad is not None}
    assert first and pfirst
    node = loss.grad_fn
    a, ws, nb = node.args, node.ws, node.nbytes
    assert bool(a.flags & L.NC_DETERMINISTIC) == deterministic
    one = torch.ones((), dtype=torch.float64, device="cuda")
    g_ro, g_rd = torch.empty_like(ro), torch.empty_like(rd)
    a.g_loss = one.data_ptr()
    a.g_rays_o, a.g_rays_d = g_ro.data_ptr(), g_rd.data_ptr()
    lib = L.load()
    L.check(lib.nc_render_backward(ctypes.byref(a), ws.data_ptr(), nb, L.raw_stream(ro.device)), "nc_render_backward")
    torch.cuda.synchronize()
    for k, f in first.items():
        assert float(f.abs().max()) > 0
        assert rel_err(g[k].grad.cpu(), (2 * f).cpu()) <= 1e-6, k
    for n, p in model.named_parameters():
        if n in pfirst:
            assert torch.equal(p.grad, pfirst[n]), n
    assert rel_err(g_ro.cpu(), ro.grad.cpu()) <= 1e-6
