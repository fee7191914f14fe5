"""Host logic of the decoder-parameter gradient modes (render_fn.param_inputs):
"autograd" hands the parameters to autograd; "direct" (the default) replaces them with
one zero-size anchor leaf and records which of them need a gradient; unknown modes are
refused."""
import pytest
import torch

from conftest import load_scene
from parity_common import build_model


def _plan():
    from nicecore.render_fn import make_plan
    bound, cbound, grids, params = load_scene()
    model = build_model(params, bound, cbound, "cpu")
    return model, make_plan("color", model)


def test_autograd_mode_passes_the_parameters():
    from nicecore.render_fn import param_inputs
    model, plan = _plan()
    spec = {}
    ins = param_inputs(spec, plan, torch.device("cpu"), "autograd")
    assert list(ins) == plan.flat_params() and "param_needs" not in spec


def test_direct_mode_anchor_and_needs():
    from nicecore.render_fn import param_inputs
    model, plan = _plan()
    flat = plan.flat_params()
    flat[3].requires_grad_(False)
    spec = {}
    ins = param_inputs(spec, plan, torch.device("cpu"), "direct")
    assert len(ins) == 1 and ins[0].numel() == 0 and ins[0].requires_grad and ins[0].is_leaf
    assert spec["param_needs"][3] is False and sum(spec["param_needs"]) == len(flat) - 1
    with torch.no_grad():
        spec = {}
        assert param_inputs(spec, plan, torch.device("cpu"), "direct") == ()
        assert not any(spec["param_needs"])


def test_default_mode_is_direct(monkeypatch):
    from nicecore import render_fn as RF
    model, plan = _plan()
    spec = {}
    ins = RF.param_inputs(spec, plan, torch.device("cpu"))
    assert RF._PARAM_GRADS == "direct" and len(ins) == 1 and "param_needs" in spec


def test_unknown_mode_refused():
    from nicecore import _lib as L
    from nicecore.render_fn import param_inputs
    model, plan = _plan()
    with pytest.raises(L.NiceCoreError):
        param_inputs({}, plan, torch.device("cpu"), "hooks")


def test_renderer_reads_config_key():
    import types
    from nicecore.renderer import Renderer
    cfg = {"rendering": {"N_samples": 32, "N_surface": 16, "N_importance": 0, "lindisp": False, "perturb": 0.,
                         "param_grads": "direct"}, "scale": 1, "occupancy": True}
    slam = types.SimpleNamespace(nice=True, bound=torch.zeros(3, 2), H=4, W=4, fx=1., fy=1., cx=1., cy=1.)
    assert Renderer(cfg, None, slam).param_grads == "direct"
    del cfg["rendering"]["param_grads"]
    assert Renderer(cfg, None, slam).param_grads is None


def test_engine_reach_of_the_anchor():
    """render_fn._engine_reaches: True for loss.backward(), False for autograd.grad(loss,
    [camera]) and backward(inputs=[...]) without the anchor -- the direct mode then
    neither computes nor writes the decoder weight gradients."""
    from nicecore.render_fn import _engine_reaches
    anchor = torch.empty(0, requires_grad=True)
    seen = []

    class F(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x, a):
            return x * 2

        @staticmethod
        def backward(ctx, g):
            seen.append(_engine_reaches(anchor))
            return g * 2, None

    cam = torch.ones(3, requires_grad=True)
    x = torch.ones(3, requires_grad=True)
    loss = F.apply(x * cam, anchor).sum()
    torch.autograd.grad(loss, [cam], retain_graph=True)
    loss.backward(inputs=[x], retain_graph=True)
    loss.backward()
    assert seen == [False, False, True]
