"""Reuse of the backward's gradient buffer (render_fn._GradBuffer): after the caller
drops last step's gradients (Mapper.py:620 / Tracker.py:135 zero_grad) the next
backward writes into the same buffer and views; while anything still references it
(kept .grad, accumulation over two backward calls, a slice held elsewhere) a fresh
buffer is taken and the old values are left untouched."""
import pytest
import torch

from parity_common import rel_err
from test_gpu_defer import _body, _leaves, _setup


def _grads(leaves):
    return [t.grad.detach().clone() if t.grad is not None else None for t in leaves]


def _same(a, b, tol=1e-6):
    for i, (x, y) in enumerate(zip(a, b)):
        assert (x is None) == (y is None), i
        if x is not None:
            assert rel_err(x.cpu(), y.cpu()) <= tol, i


@pytest.mark.gpu
def test_buffer_reused_after_grads_dropped():
    sc, g, model, ro, rd, gt, gtc, r = _setup()
    leaves = _leaves(g, model, ro, rd)
    p0 = model.color_decoder.output_linear.weight  # a decoder the color stage trains
    _body(r, g, model, ro, rd, gt, gtc, None)
    ref = _grads(leaves)
    ptr = p0.grad.data_ptr()
    gptr = g["grid_fine"].grad.data_ptr()
    _body(r, g, model, ro, rd, gt, gtc, None)  # sets every .grad to None first
    assert p0.grad.data_ptr() == ptr and g["grid_fine"].grad.data_ptr() == gptr
    _same(_grads(leaves), ref)


@pytest.mark.gpu
def test_accumulation_takes_a_fresh_buffer():
    sc, g, model, ro, rd, gt, gtc, r = _setup()
    leaves = _leaves(g, model, ro, rd)
    _body(r, g, model, ro, rd, gt, gtc, None)
    ref = _grads(leaves)
    # second backward without dropping the gradients: AccumulateGrad adds into them
    d, u, c, L = r.render_batch_loss(g, model, rd, ro, "cuda", "color", gt, gtc, loss="mapper", color_term=True)
    L.backward()
    _same(_grads(leaves), [2 * x if x is not None else None for x in ref], tol=2e-6)


@pytest.mark.gpu
def test_held_slice_is_not_overwritten():
    sc, g, model, ro, rd, gt, gtc, r = _setup()
    p0 = model.color_decoder.output_linear.weight  # a decoder the color stage trains
    _body(r, g, model, ro, rd, gt, gtc, None)
    held = p0.grad.view(-1)[:8]
    before = held.clone()
    gh = g["grid_fine"].grad[0, :, 0, 0, 0]
    gbefore = gh.clone()
    ro.data.mul_(1.001)  # different rays: a reused buffer would change the held values
    _body(r, g, model, ro, rd, gt, gtc, None)
    torch.cuda.synchronize()
    assert torch.equal(held, before) and torch.equal(gh, gbefore)
    assert p0.grad.data_ptr() != held.data_ptr()


def _body_mode(r, g, model, ro, rd, gt, gtc, mode):
    for t in _leaves(g, model, ro, rd):
        t.grad = None
    r.param_grads = mode
    d, u, c, L = r.render_batch_loss(g, model, rd, ro, "cuda", "color", gt, gtc, loss="mapper", color_term=True)
    L.backward()
    return L


@pytest.mark.gpu
def test_direct_param_grads_match_autograd():
    """param_grads="direct" (render_fn.param_inputs): the decoder weight gradients are
    bit-identical to the autograd mode's (same kernels, fixed reduction order), grid /
    ray gradients to the float-atomic tolerance; a second backward adds into .grad."""
    sc, g, model, ro, rd, gt, gtc, r = _setup()
    leaves = _leaves(g, model, ro, rd)
    _body_mode(r, g, model, ro, rd, gt, gtc, "autograd")
    ref = _grads(leaves)
    _body_mode(r, g, model, ro, rd, gt, gtc, "direct")
    got = _grads(leaves)
    n0, n1 = len(g), len(g) + len(list(model.parameters()))
    for i, (a, b) in enumerate(zip(got, ref)):
        assert (a is None) == (b is None), i
        if a is not None:
            if n0 <= i < n1:
                assert torch.equal(a, b), i
            else:
                assert rel_err(a.cpu(), b.cpu()) <= 1e-6, i
    d, u, c, L = r.render_batch_loss(g, model, rd, ro, "cuda", "color", gt, gtc, loss="mapper", color_term=True)
    L.backward()
    _same(_grads(leaves), [2 * x if x is not None else None for x in ref], tol=2e-6)


@pytest.mark.gpu
def test_direct_param_grads_graph_replay():
    from nicecore.graph import GraphedStep
    sc, g, model, ro, rd, gt, gtc, r = _setup()
    leaves = _leaves(g, model, ro, rd)
    _body_mode(r, g, model, ro, rd, gt, gtc, "autograd")
    ref = _grads(leaves)
    step = GraphedStep(lambda: _body_mode(r, g, model, ro, rd, gt, gtc, "direct"))
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    _same(_grads(leaves), ref)


@pytest.mark.gpu
def test_direct_mode_autograd_grad_leaves_params_alone():
    """param_grads="direct" under torch.autograd.grad(loss, [rays]) and backward(inputs=
    [grid]): the decoder parameters are not among the requested gradients, so their .grad
    stays None (k_mlp_dw is not launched), as autograd would leave it; the requested
    gradients equal the full backward's."""
    sc, g, model, ro, rd, gt, gtc, r = _setup()
    leaves = _leaves(g, model, ro, rd)
    _body_mode(r, g, model, ro, rd, gt, gtc, "direct")
    full = _grads(leaves)
    n0, n1 = len(g), len(g) + len(list(model.parameters()))
    for t in leaves:
        t.grad = None
    d, u, c, L = r.render_batch_loss(g, model, rd, ro, "cuda", "color", gt, gtc, loss="mapper", color_term=True)
    gro, grd = torch.autograd.grad(L, [ro, rd])
    assert all(t.grad is None for t in leaves)
    assert rel_err(gro.cpu(), full[-2].cpu()) <= 1e-6 and rel_err(grd.cpu(), full[-1].cpu()) <= 1e-6
    d, u, c, L = r.render_batch_loss(g, model, rd, ro, "cuda", "color", gt, gtc, loss="mapper", color_term=True)
    L.backward(inputs=[g["grid_fine"]])
    got = _grads(leaves)
    for i, t in enumerate(got):
        if n0 <= i < n1:
            assert t is None, i
    assert rel_err(g["grid_fine"].grad.cpu(), full[list(g).index("grid_fine")].cpu()) <= 1e-6
