"""GraphedStep and the autograd engine's streams.

Round 4's GPU run crashed the test process in ``torch.cuda.graphs.capture_end``
(``GraphedStep.__init__``) for a body that kept its undetached loss in an enclosing dict
(``out["loss"] = loss``) after eager calls of the same body on the default stream.  The
cause (nicecore/graph.py docstring): every call's graph kept the previous
call's gradient accumulators alive, so the captured backward reached accumulators created
on the default stream, and the engine made that stream wait on the capture.  GraphedStep
now warms up and captures on one stream and refuses that pattern with an error; the body
of the round-4 test is restored here as the regression case.  The loop shape it follows is
the reference's Tracker step (src/Tracker.py:113-135: ``loss.backward()`` at :132, the loss
still alive for ``return loss.item()`` at :135)."""
import pytest
import torch

from parity_common import make_renderer, rel_err
from test_gpu_ray_mask import _case, _leaves


def _setup(n_rays=256, seed=66):
    sc, grids, params, ro, rd, dep, col, keep = _case(n_rays, seed=seed)
    model, g, ro_g, rd_g = _leaves(sc, grids, params, ro, rd, "ba")
    r = make_renderer(sc.bound)
    gt, gtc = dep.cuda(), col.cuda()
    mask = keep.cuda().clone()
    leaves = [g[k] for k in ("grid_middle", "grid_fine", "grid_color")] + \
        [p for n, p in model.named_parameters() if not n.startswith("coarse_decoder.")] + [ro_g, rd_g]
    out = {}

    def body():  # the round-4 body: the undetached loss kept in an enclosing dict
        for t in leaves:
            t.grad = None
        d, u, c, loss = r.render_batch_loss(g, model, rd_g, ro_g, "cuda", "color", gt, gtc, loss="mapper",
                                            w_color_loss=0.2, color_term=True, ray_mask=mask)
        loss.backward()
        out["loss"] = loss
        return loss

    masks = [keep, torch.roll(keep, 7), torch.ones_like(keep)]
    return body, out, leaves, mask, masks


def _replay_matches(step, eager, masks, mask, leaves):
    for (l0, g0), mk in zip(eager, masks):
        mask.copy_(mk.cuda())
        loss = step()
        torch.cuda.synchronize()
        assert abs(float(loss) - l0) <= 1e-6 * max(abs(l0), 1.0)
        for t, gr in zip(leaves, g0):
            assert rel_err(t.grad.cpu(), gr.cpu()) <= 1e-6


@pytest.mark.gpu
def test_graphed_step_refuses_accumulators_of_an_older_graph():
    """The exact round-4 sequence: eager calls of the loss-keeping body, then GraphedStep.
    It must raise (naming the cause), not crash; once the old loss is dropped the same body
    captures and every replay equals the eager masked step."""
    from nicecore._lib import NiceCoreError
    from nicecore.graph import GraphedStep
    body, out, leaves, mask, masks = _setup()
    eager = []
    for mk in masks:
        mask.copy_(mk.cuda())
        body()
        eager.append((float(out["loss"]), [t.grad.detach().clone() for t in leaves]))
    with pytest.raises(NiceCoreError, match="alive before the GraphedStep was built"):
        GraphedStep(body)
    out.clear()  # drop the eager graph: its accumulators die with it
    step = GraphedStep(body)  # the body still keeps its own loss across warm-up and capture
    _replay_matches(step, eager, masks, mask, leaves)
    # eager calls after the capture (accumulators now on the capture stream, outside capture)
    mask.copy_(masks[0].cuda())
    body()
    torch.cuda.synchronize()
    assert abs(float(out["loss"]) - eager[0][0]) <= 1e-6 * max(abs(eager[0][0]), 1.0)


@pytest.mark.gpu
def test_graphed_step_body_keeping_its_loss_without_prior_eager_calls():
    """A body that keeps its loss for logging and is captured before any eager call: the
    accumulators are created by the warm-up on the capture stream, nothing is refused."""
    from nicecore.graph import GraphedStep
    body, out, leaves, mask, masks = _setup(seed=67)
    step = GraphedStep(body)
    replayed = []
    for mk in masks:
        mask.copy_(mk.cuda())
        loss = step()
        torch.cuda.synchronize()
        replayed.append((float(loss), [t.grad.detach().clone() for t in leaves]))
    out.clear()
    for (l1, g1), mk in zip(replayed, masks):  # eager references, the graph dropped each time
        mask.copy_(mk.cuda())
        body()
        torch.cuda.synchronize()
        l0 = float(out["loss"])
        assert abs(l1 - l0) <= 1e-6 * max(abs(l0), 1.0)
        for t, gr in zip(leaves, g1):
            assert rel_err(gr.cpu(), t.grad.cpu()) <= 1e-6
        out.clear()
