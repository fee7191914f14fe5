"""The fused rendering loss (k_loss + its derivatives folded into k_composite_bwd)
vs the oracle's statement of the same loss (oracle/nice_oracle.py mapper_loss /
tracker_loss, Mapper.py:603-612, Tracker.py:117-131) evaluated by autograd on the
unfused render outputs.

Tolerances:
  * render outputs: bit-identical (same kernels);
  * loss value: 1e-12 relative for the float64 depth term; the float32 colour sum
    is accumulated in float64 and rounded once, the reference's float32 sum is
    pairwise, so the colour term is compared to 1e-6 relative;
  * every gradient: 1e-6 of its max-abs (the upstream derivatives are the same
    expressions; the residual is the float atomics of the grid scatter).
Against the reference's own render outputs (golden) the loss agrees to the render
tolerance (2e-5); the loss value itself has no reference fixture (DESIGN.md:
"parity unpinned" for the loss term).
"""
import pytest
import torch

from conftest import load_case, load_scene
from parity_common import build_model, case_stage, make_renderer, rel_err
from oracle import nice_oracle as O

LOSSES = [  # (loss, color_term, handle_dynamic)
    ("mapper", False, False), ("mapper", True, False),
    ("tracker", True, True), ("tracker", False, False), ("tracker", True, False), ("tracker", False, True)]


def _oracle_loss(kind, d, v, c, gt, gtc, color_term, dyn):
    if kind == "mapper":
        return O.mapper_loss(d, c, gt, gtc, 0.2, color_term)
    return O.tracker_loss(d, v, c, gt, gtc, 0.5, color_term, dyn)


def _setup(case, want_rays=True):
    bound, cbound, grids, params = load_scene()
    rec = load_case(case)
    stage, _ = case_stage(case)
    model = build_model(params, bound, cbound, "cuda")
    g = {k: v.cuda().requires_grad_(True) for k, v in grids.items()}
    ro = rec["rays_o"].cuda().requires_grad_(want_rays)
    rd = rec["rays_d"].cuda().requires_grad_(want_rays)
    return rec, stage, model, g, ro, rd, make_renderer(bound)


def _grads(model, g, ro, rd):
    out = {}
    for k, v in g.items():
        if v.grad is not None:
            out["grid/" + k] = v.grad.detach().clone()
            v.grad = None
    for n, p in model.named_parameters():
        if p.grad is not None:
            out["param/" + n] = p.grad.detach().clone()
            p.grad = None
    for k, t in (("rays_o", ro), ("rays_d", rd)):
        if t.grad is not None:
            out[k] = t.grad.detach().clone()
            t.grad = None
    return out


def _compare_fused_unfused(r, stage, model, g, ro, rd, gt, gtc, kind, color_term, dyn, dmax=None):
    d1, v1, c1, L1 = r.render_batch_loss(g, model, rd, ro, "cuda", stage, gt, gtc, loss=kind,
                                         w_color_loss=0.2 if kind == "mapper" else 0.5,
                                         color_term=color_term, handle_dynamic=dyn, depth_max=dmax)
    L1.backward()
    G1 = _grads(model, g, ro, rd)
    d2, v2, c2 = r.render_batch_ray(g, model, rd, ro, "cuda", stage, gt, depth_max=dmax)
    L2 = _oracle_loss(kind, d2, v2, c2, gt, gtc, color_term, dyn)
    L2.backward()
    G2 = _grads(model, g, ro, rd)
    assert torch.equal(d1, d2) and torch.equal(v1, v2) and torch.equal(c1, c2)
    assert L1.dtype == torch.float64 and L1.shape == ()
    a, b = float(L1.detach()), float(L2.detach())
    tol = (1e-6 if color_term else 1e-12) * (abs(b) + 1e-30)
    assert abs(a - b) <= tol, (a, b)
    assert set(G1) == set(G2), (sorted(G1), sorted(G2))
    bad = {k: rel_err(G1[k].cpu(), G2[k].cpu()) for k in G1 if rel_err(G1[k].cpu(), G2[k].cpu()) > 1e-6}
    assert not bad, bad
    return a, (d1, v1, c1)


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["color_depth", "fine_depth", "middle_depth"])
@pytest.mark.parametrize("kind,color_term,dyn", LOSSES)
def test_fused_loss_matches_oracle(case, kind, color_term, dyn):
    rec, stage, model, g, ro, rd, r = _setup(case)
    gt, gtc = rec["gt_depth"].cuda(), rec["gt_color"].cuda()
    loss, _ = _compare_fused_unfused(r, stage, model, g, ro, rd, gt, gtc, kind, color_term, dyn)
    # the same loss statement on the REFERENCE's render outputs (golden)
    ref = _oracle_loss(kind, rec["depth"], rec["var"], rec["color"], rec["gt_depth"], rec["gt_color"],
                       color_term, dyn)
    assert abs(loss - float(ref)) <= 2e-5 * abs(float(ref)) + 1e-9


@pytest.mark.gpu
@pytest.mark.parametrize("n_rays", [1, 2, 1000, 1024, 1025, 4099])
@pytest.mark.parametrize("kind,color_term,dyn", [("tracker", True, True), ("mapper", True, False)])
def test_fused_loss_room0_sizes(n_rays, kind, color_term, dyn):
    """Replica room0 scene at the mapper's / tracker's batch sizes and beyond one ray
    per thread of k_loss (1024, 1025, 4099 > 4 x 1024): median radix select, strided
    sums."""
    from test_gpu_parity import _room0_case
    sc, grids, params, ro, rd, dep = _room0_case(n_rays, "color", seed=11)
    model = build_model(params, sc.bound, sc.bound * 2, "cuda")
    g = {k: v.cuda().requires_grad_(True) for k, v in grids.items()}
    ro = ro.cuda().requires_grad_(True)
    rd = rd.cuda().requires_grad_(True)
    gt = dep.cuda()
    gtc = torch.rand(n_rays, 3, generator=torch.Generator().manual_seed(3)).cuda()
    r = make_renderer(sc.bound, H=sc.H, W=sc.W)
    _compare_fused_unfused(r, "color", model, g, ro, rd, gt, gtc, kind, color_term, dyn)


@pytest.mark.gpu
def test_fix_fine_color_decoder_only():
    """The Mapper's fix_fine (configs/nice_slam.yaml:62, Mapper.py:416-424): only the color
    decoder requires grad.  k_mlp_dw then runs all its workgroups on the color decoder
    (nc_abi.hip fill_mlp); its gradient equals the all-decoders run's (1e-6 of max-abs:
    the slab partition, so the summation order, differs) and no frozen decoder gets one."""
    from test_gpu_parity import _room0_case
    sc, grids, params, ro, rd, dep = _room0_case(1000, "color", seed=5)
    model = build_model(params, sc.bound, sc.bound * 2, "cuda")
    g = {k: v.cuda().requires_grad_(True) for k, v in grids.items()}
    ro = ro.cuda().requires_grad_(True)
    rd = rd.cuda().requires_grad_(True)
    gt = dep.cuda()
    gtc = torch.rand(1000, 3, generator=torch.Generator().manual_seed(4)).cuda()
    r = make_renderer(sc.bound, H=sc.H, W=sc.W)
    L = r.render_batch_loss(g, model, rd, ro, "cuda", "color", gt, gtc, loss="mapper", color_term=True)[3]
    L.backward()
    full = _grads(model, g, ro, rd)
    for n in ("coarse", "middle", "fine"):
        for p in getattr(model, n + "_decoder").parameters():
            p.requires_grad_(False)
    _compare_fused_unfused(r, "color", model, g, ro, rd, gt, gtc, "mapper", True, False)
    L = r.render_batch_loss(g, model, rd, ro, "cuda", "color", gt, gtc, loss="mapper", color_term=True)[3]
    L.backward()
    part = _grads(model, g, ro, rd)
    assert all(not k.startswith("param/") or k.startswith("param/color_decoder.") for k in part), sorted(part)
    assert any(k.startswith("param/color_decoder.") for k in part)
    bad = {k: rel_err(part[k].cpu(), full[k].cpu()) for k in part if rel_err(part[k].cpu(), full[k].cpu()) > 1e-6}
    assert not bad, bad


@pytest.mark.gpu
def test_fused_loss_sharded_depth_max():
    """The data-parallel form: a supplied depth_max (the all-reduced max) with the loss."""
    rec, stage, model, g, ro, rd, r = _setup("color_depth")
    gt, gtc = rec["gt_depth"].cuda(), rec["gt_color"].cuda()
    dmax = gt.max().reshape(1) * 1.5
    _compare_fused_unfused(r, stage, model, g, ro, rd, gt, gtc, "mapper", True, False, dmax=dmax)


@pytest.mark.gpu
def test_fused_loss_tracker_rays_only():
    """Tracker mode: decoders and grids frozen, gradient to the rays only."""
    rec, stage, model, g, ro, rd, r = _setup("color_depth")
    for p in model.parameters():
        p.requires_grad_(False)
    for v in g.values():
        v.requires_grad_(False)
    gt, gtc = rec["gt_depth"].cuda(), rec["gt_color"].cuda()
    _compare_fused_unfused(r, stage, model, g, ro, rd, gt, gtc, "tracker", True, True)


@pytest.mark.gpu
def test_fused_loss_empty_batch():
    bound, cbound, grids, params = load_scene()
    model = build_model(params, bound, cbound, "cuda")
    g = {k: v.cuda() for k, v in grids.items()}
    r = make_renderer(bound)
    z = torch.zeros(0, 3, device="cuda")
    d, v, c, L = r.render_batch_loss(g, model, z, z, "cuda", "color", torch.zeros(0, device="cuda"),
                                     torch.zeros(0, 3, device="cuda"), loss="mapper", color_term=True)
    assert d.shape == (0,) and float(L) == 0.0


@pytest.mark.gpu
def test_fused_loss_upstream_scale():
    """A non-unit upstream gradient on the loss scales every derivative (2 * loss)."""
    rec, stage, model, g, ro, rd, r = _setup("color_depth")
    gt, gtc = rec["gt_depth"].cuda(), rec["gt_color"].cuda()
    d, v, c, L = r.render_batch_loss(g, model, rd, ro, "cuda", stage, gt, gtc, loss="mapper", color_term=True)
    (2.0 * L).backward()
    G2 = _grads(model, g, ro, rd)
    d, v, c, L = r.render_batch_loss(g, model, rd, ro, "cuda", stage, gt, gtc, loss="mapper", color_term=True)
    L.backward()
    G1 = _grads(model, g, ro, rd)
    for k in G1:
        assert rel_err(G2[k].cpu(), 2.0 * G1[k].cpu()) <= 1e-6, k


@pytest.mark.gpu
def test_fused_loss_with_output_gradients():
    """The mapper loss's forward writes d raw for d loss = 1 (k_composite_fwd_loss); a
    backward that also receives depth / colour gradients runs k_composite_bwd on the
    forward's loss coefficients instead: both must equal the unfused statement."""
    rec, stage, model, g, ro, rd, r = _setup("color_depth")
    gt, gtc = rec["gt_depth"].cuda(), rec["gt_color"].cuda()
    d1, v1, c1, L1 = r.render_batch_loss(g, model, rd, ro, "cuda", stage, gt, gtc, loss="mapper", color_term=True)
    (L1 + 0.5 * d1.sum() + (c1 * c1).sum()).backward()
    G1 = _grads(model, g, ro, rd)
    d2, v2, c2 = r.render_batch_ray(g, model, rd, ro, "cuda", stage, gt)
    L2 = _oracle_loss("mapper", d2, v2, c2, gt, gtc, True, False)
    (L2 + 0.5 * d2.sum() + (c2 * c2).sum()).backward()
    G2 = _grads(model, g, ro, rd)
    assert set(G1) == set(G2)
    bad = {k: rel_err(G1[k].cpu(), G2[k].cpu()) for k in G1 if rel_err(G1[k].cpu(), G2[k].cpu()) > 1e-6}
    assert not bad, bad


@pytest.mark.gpu
def test_fused_loss_retain_graph_second_backward():
    """A backward with output gradients runs k_composite_bwd (d raw of loss + depth terms);
    on a retained graph a later backward of the loss alone takes the fused path again and
    must still find the forward's d raw for d loss = 1 (not the first backward's): it equals
    the loss-only backward of a fresh render."""
    rec, stage, model, g, ro, rd, r = _setup("color_depth")
    gt, gtc = rec["gt_depth"].cuda(), rec["gt_color"].cuda()
    d1, v1, c1, L1 = r.render_batch_loss(g, model, rd, ro, "cuda", stage, gt, gtc, loss="mapper", color_term=True)
    (L1 + 0.5 * d1.sum() + (c1 * c1).sum()).backward(retain_graph=True)
    _grads(model, g, ro, rd)
    L1.backward()
    G1 = _grads(model, g, ro, rd)
    L2 = r.render_batch_loss(g, model, rd, ro, "cuda", stage, gt, gtc, loss="mapper", color_term=True)[3]
    L2.backward()
    G2 = _grads(model, g, ro, rd)
    assert set(G1) == set(G2)
    bad = {k: rel_err(G1[k].cpu(), G2[k].cpu()) for k in G1 if rel_err(G1[k].cpu(), G2[k].cpu()) > 1e-6}
    assert not bad, bad


@pytest.mark.gpu
def test_no_weight_grad_flag_is_enforced(monkeypatch):
    """NC_NO_WEIGHT_GRAD(kind) (include/nicecore.h) spares the forward's activation records
    of a decoder; a backward that then asks for that decoder's weight gradient must fail
    loudly instead of reading records that were never written."""
    from nicecore import _lib as L
    from nicecore import render_fn as RF
    rec, stage, model, g, ro, rd, r = _setup("color_depth")
    gt, gtc = rec["gt_depth"].cuda(), rec["gt_color"].cuda()
    orig = RF._flags
    monkeypatch.setattr(RF, "_flags", lambda ctx, spec, ci=(): orig(ctx, spec, ci) | L.NC_NO_WEIGHT_GRAD(3))
    L_ = r.render_batch_loss(g, model, rd, ro, "cuda", stage, gt, gtc, loss="mapper", color_term=True)[3]
    with pytest.raises(L.NiceCoreError, match="NC_NO_WEIGHT_GRAD"):
        L_.backward()


@pytest.mark.gpu
@pytest.mark.parametrize("color_term", [True, False])
def test_fused_loss_value_fixed_order(color_term):
    """k_composite_fwd_loss sums the loss in a fixed order (per-workgroup partials, the last
    workgroup adds them in block order and applies w_color once to the float32 colour
    total, as k_loss): the value is bit-identical from run to run and equals the
    three-kernel path's (NC_DETERMINISTIC: k_loss) to float64 rounding for the depth term,
    1e-6 relative with the float32 colour term."""
    from nicecore import ops
    from test_gpu_parity import _room0_case
    n = 5000  # 313 workgroups of 16 rays
    sc, grids, params, ro, rd, dep = _room0_case(n, "color", seed=12)
    model = build_model(params, sc.bound, sc.bound * 2, "cuda")
    g = {k: v.cuda().requires_grad_(True) for k, v in grids.items()}
    c = dict(g)
    ro, rd, gt = ro.cuda(), rd.cuda(), dep.cuda()
    gtc = torch.rand(n, 3, generator=torch.Generator().manual_seed(4)).cuda()

    def loss(det):
        out = ops.render_rays_loss(model, c, ro, rd, sc.bound, "color", gt, loss="mapper", target_color=gtc,
                                   w_color=0.2, color_term=color_term, deterministic=det)
        return float(out[3].detach())
    vals = [loss(None) for _ in range(4)]
    assert len(set(vals)) == 1, vals
    ref = loss(True)
    tol = (1e-6 if color_term else 1e-13) * abs(ref)
    assert abs(vals[0] - ref) <= tol, (vals[0], ref)
