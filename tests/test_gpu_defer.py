"""Split backward for data-parallel overlap (render_fn.DeferParamGrads,
NC_DEFER_PARAM_GRADS + nc_render_backward_params, ABI v7): the backward produces the
grid and ray gradients, the decoder weight gradients come from a second call.  The
split must not change any gradient: weight gradients bit-identical (same kernels, slab
reduction in a fixed order), grid / ray gradients to the float-atomic tolerance (1e-6
of max-abs), eagerly and as two hipGraph captures (bench.py N > 1)."""
import pytest
import torch

from parity_common import build_model, make_renderer, rel_err
from test_gpu_parity import _room0_case


def _setup():
    sc, grids, params, ro, rd, dep = _room0_case(300, "color", seed=21)
    model = build_model(params, sc.bound, sc.bound * 2, "cuda")
    g = {k: v.cuda().contiguous(memory_format=torch.channels_last_3d).requires_grad_(True) for k, v in grids.items()}
    ro, rd = ro.cuda().requires_grad_(True), rd.cuda().requires_grad_(True)
    gtc = torch.rand(300, 3, generator=torch.Generator().manual_seed(2)).cuda()
    return sc, g, model, ro, rd, dep.cuda(), gtc, make_renderer(sc.bound, H=sc.H, W=sc.W)


def _leaves(g, model, ro, rd):
    return list(g.values()) + list(model.parameters()) + [ro, rd]


def _body(r, g, model, ro, rd, gt, gtc, defer):
    for t in _leaves(g, model, ro, rd):
        t.grad = None
    if defer is not None:
        defer.clear()
    d, u, c, L = r.render_batch_loss(g, model, rd, ro, "cuda", "color", gt, gtc, loss="mapper",
                                     color_term=True, defer_param_grads=defer)
    L.backward()
    return L


def _check(got, ref, leaves, n_params_from):
    for i, (a, b) in enumerate(zip(got, ref)):
        assert (a is None) == (b is None), i
        if a is None:
            continue
        if n_params_from[0] <= i < n_params_from[1]:
            assert torch.equal(a, b), i  # decoder weight gradients: same order of summation
        else:
            assert rel_err(a.cpu(), b.cpu()) <= 1e-6, i


@pytest.mark.gpu
def test_deferred_weight_gradients_eager():
    from nicecore.render_fn import DeferParamGrads
    sc, g, model, ro, rd, gt, gtc, r = _setup()
    leaves = _leaves(g, model, ro, rd)
    _body(r, g, model, ro, rd, gt, gtc, None)
    ref = [t.grad.detach().clone() if t.grad is not None else None for t in leaves]
    defer = DeferParamGrads()
    _body(r, g, model, ro, rd, gt, gtc, defer)
    assert all(p.grad is None for p in model.parameters())  # not yet
    assert g["grid_fine"].grad is not None and ro.grad is not None
    defer.run()
    got = [t.grad.detach().clone() if t.grad is not None else None for t in leaves]
    _check(got, ref, leaves, (4, 4 + len(list(model.parameters()))))


@pytest.mark.gpu
def test_deferred_weight_gradients_two_graphs():
    from nicecore.graph import GraphedStep
    from nicecore.render_fn import DeferParamGrads
    sc, g, model, ro, rd, gt, gtc, r = _setup()
    leaves = _leaves(g, model, ro, rd)
    _body(r, g, model, ro, rd, gt, gtc, None)
    ref = [t.grad.detach().clone() if t.grad is not None else None for t in leaves]
    defer = DeferParamGrads()
    g1 = GraphedStep(lambda: _body(r, g, model, ro, rd, gt, gtc, defer))
    g2 = GraphedStep(defer.run)
    for _ in range(2):
        g1()
        g2()
    torch.cuda.synchronize()
    got = [t.grad.detach().clone() if t.grad is not None else None for t in leaves]
    _check(got, ref, leaves, (4, 4 + len(list(model.parameters()))))


@pytest.mark.gpu
def test_split_allreduce_two_gloo_ranks(tmp_path):
    """Two gloo ranks (subprocesses on one GPU) each render half the batch and run the
    split exchange: the reduced grid and decoder gradients equal the single-process
    gradient of the whole batch (1e-5 of max-abs: float atomics + a different sum order)."""
    import os
    import subprocess
    import sys
    from conftest import REPO
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29641", HSA_ENABLE_IPC_MODE_LEGACY="0")
    procs = [subprocess.Popen([sys.executable, os.path.join(REPO, "tests", "defer_dist_worker.py"), str(tmp_path)],
                              env=dict(env, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r))) for r in range(2)]
    for p in procs:
        assert p.wait(timeout=110) == 0
    outs = [torch.load(tmp_path / f"defer_rank{r}.pt", weights_only=True) for r in range(2)]
    sc, g, model, ro, rd, gt, gtc, r = _setup()
    _body(r, g, model, ro, rd, gt, gtc, None)
    ref = {k: v.grad.cpu() for k, v in g.items() if v.grad is not None}
    ref.update({"param/" + n: p.grad.cpu() for n, p in model.named_parameters() if p.grad is not None})
    assert set(outs[0]) == set(ref) and len(ref) > 4
    for k in ref:
        assert torch.equal(outs[0][k], outs[1][k]), k
        assert rel_err(outs[0][k], ref[k]) <= 1e-5, (k, rel_err(outs[0][k], ref[k]))
