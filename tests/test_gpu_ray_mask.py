"""Per-ray validity mask (ABI v10 ``nc_render_args.ray_valid``; ``ray_mask=`` of
render_batch_ray / render_batch_loss): the callers' bbox pre-filter
(src/Tracker.py:100-111, src/Mapper.py:580-596) without the boolean-index compaction.

A masked render of N rays must equal rendering the compacted batch rays[mask]:
  * kept rays' depth / uncertainty / colour and ray gradients bit-identical (every point's
    decoder chains and every ray's compositing are independent of the other rays; the
    batch-global max(gt_depth) is taken over the kept rays, Renderer.py:157, :194);
  * the loss (mapper, tracker with handle_dynamic's median over the kept rays): the float64
    depth term to 1e-12; with the float32 colour term to 1e-6 relative (its per-workgroup
    partial sums group the rays differently in the two batches; tests/test_gpu_loss.py);
  * grid and decoder-parameter gradients to 1e-6 of max-abs (float atomics / a different
    point blocking of the weight-gradient sums);
  * dropped rays: outputs and ray gradients exactly 0.
and the compacted batch itself is held to the CPU oracle (float64 truth scoring)."""
import pytest
import torch

from parity_common import build_model, make_renderer, oracle_render_grads, rel_err, score_vs_truth

DROP_FRAC = 0.25


def _case(n_rays, seed=21, std=0.3):
    from nicecore import decoder as D
    from nicecore import scene as S
    sc = S.make_scene("replica_room0")
    grids = S.init_grids(sc.shapes, generator=torch.Generator().manual_seed(seed),
                         std={k: std for k in S.GRID_STD})
    m = D.build_default_nice(seed=seed)
    with torch.no_grad():
        m.middle_decoder.output_linear.bias.fill_(-0.5)
        m.fine_decoder.output_linear.bias.fill_(-0.4)
    params = {k: v.detach().clone() for k, v in m.named_parameters()}
    ro, rd, dep, col = S.synth_rays(sc, n_rays, seed=seed + 1)
    # push DROP_FRAC of the rays' target depth past the bound's exit: the callers' filter
    # (t_exit >= gt_depth) rejects them; a few of them get the largest depth of the batch,
    # so a compaction-unaware max(gt_depth) would differ
    gen = torch.Generator().manual_seed(seed + 2)
    drop = torch.rand(n_rays, generator=gen) < DROP_FRAC
    t_exit = S.ray_exit_t(sc.bound, ro, rd).float()
    dep = torch.where(drop, t_exit * 1.5 + 0.5, dep)
    keep = S.ray_exit_t(sc.bound, ro, rd) >= dep.double()
    assert torch.equal(keep, ~drop)
    return sc, grids, params, ro, rd, dep, col, keep


def _leaves(sc, grids, params, ro, rd, mode):
    model = build_model(params, sc.bound, sc.bound * 2, "cuda")
    ba = mode == "ba"
    for p in model.parameters():
        p.requires_grad_(ba)
    g = {k: v.cuda().contiguous(memory_format=torch.channels_last_3d).requires_grad_(ba) for k, v in grids.items()}
    return model, g, ro.cuda().requires_grad_(True), rd.cuda().requires_grad_(True)


def _grads(model, g, ro, rd):
    out = {"grad/rays_o": ro.grad, "grad/rays_d": rd.grad}
    for k, v in g.items():
        if v.grad is not None:
            out["grad/" + k] = v.grad
    for n, p in model.named_parameters():
        if p.grad is not None:
            out["grad/param/" + n] = p.grad
    return {k: v.detach().cpu() for k, v in out.items() if v is not None}


def _run(sc, grids, params, ro, rd, dep, col, mask, mode, fused):
    """(outputs, loss, grads) of one render + loss + backward; ``mask``: ray_mask, or
    None to render the rays as given."""
    model, g, ro_g, rd_g = _leaves(sc, grids, params, ro, rd, mode)
    r = make_renderer(sc.bound)
    gt, gtc = dep.cuda(), col.cuda()
    m = mask.cuda() if mask is not None else None
    if fused:
        kw = (dict(loss="mapper", w_color_loss=0.2, color_term=True) if mode == "ba" else
              dict(loss="tracker", w_color_loss=0.5, color_term=True, handle_dynamic=True))
        d, u, c, loss = r.render_batch_loss(g, model, rd_g, ro_g, "cuda", "color", gt, gtc, **kw, ray_mask=m)
    else:  # the reference's Python loss (Mapper.py:603-612) over the kept rays
        d, u, c = r.render_batch_ray(g, model, rd_g, ro_g, "cuda", "color", gt, ray_mask=m)
        keep = m if m is not None else torch.ones_like(gt, dtype=torch.bool)
        dm = (gt > 0) & keep
        loss = (gt.double() - d).abs()[dm].sum() + 0.2 * (gtc - c).abs()[keep].sum()
    loss.backward()
    outs = {"depth": d.detach().cpu(), "var": u.detach().cpu(), "color": c.detach().cpu()}
    return outs, float(loss), _grads(model, g, ro_g, rd_g)


@pytest.mark.gpu
@pytest.mark.parametrize("mode,fused", [("ba", True), ("ba", False), ("tracker", True)])
@pytest.mark.parametrize("n_rays", [600, 5000])
def test_masked_equals_compacted(mode, fused, n_rays):
    """5,000 rays (ScanNet tracking's pixel count, the Mapper's BA batch size) take the
    masked paths that only run above 4,096 rays -- k_depth_max's kept-ray filter and k_loss's
    uncached median over the kept rays -- while the ~3,750-ray compacted batch takes the
    cached ones."""
    sc, grids, params, ro, rd, dep, col, keep = _case(n_rays)
    assert DROP_FRAC * 0.8 < float((~keep).float().mean()) < DROP_FRAC * 1.2
    om, lm, gm = _run(sc, grids, params, ro, rd, dep, col, keep, mode, fused)
    oc, lc, gc = _run(sc, grids, params, ro[keep], rd[keep], dep[keep], col[keep], None, mode, fused)
    for k in ("depth", "var", "color"):
        assert torch.equal(om[k][keep], oc[k]), k
        assert not bool(om[k][~keep].any()), k  # dropped rays report 0
    assert abs(lm - lc) <= 1e-6 * max(abs(lc), 1.0), (lm, lc)  # colour term on: test_gpu_loss.py's bound
    for k in ("grad/rays_o", "grad/rays_d"):
        assert torch.equal(gm[k][keep], gc[k]), k
        assert not bool(gm[k][~keep].any()), k
    assert set(gm) == set(gc), set(gm) ^ set(gc)
    for k in gm:
        if k.startswith("grad/rays"):
            continue
        assert rel_err(gm[k], gc[k]) <= 1e-6, (k, rel_err(gm[k], gc[k]))


@pytest.mark.gpu
def test_masked_render_against_oracle_on_compacted_batch():
    """The masked HIP render scored against the oracle on rays[mask] (float64 truth)."""
    sc, grids, params, ro, rd, dep, col, keep = _case(300, seed=33)
    model, g, ro_g, rd_g = _leaves(sc, grids, params, ro, rd, "ba")
    r = make_renderer(sc.bound)
    gen = torch.Generator().manual_seed(5)
    n = ro.shape[0]
    up = (torch.randn(n, generator=gen, dtype=torch.float64), torch.randn(n, generator=gen, dtype=torch.float64),
          torch.randn(n, 3, generator=gen))
    d, u, c = r.render_batch_ray(g, model, rd_g, ro_g, "cuda", "color", dep.cuda(), ray_mask=keep.cuda())
    torch.autograd.backward([d, u, c], [t.cuda() for t in up])
    got = {"depth": d.detach().cpu()[keep], "var": u.detach().cpu()[keep], "color": c.detach().cpu()[keep]}
    gg = _grads(model, g, ro_g, rd_g)
    got.update({k: (v[keep] if k.startswith("grad/rays") else v) for k, v in gg.items()})
    dec_b = {"coarse": sc.bound * 2, "middle": sc.bound, "fine": sc.bound, "color": sc.bound}
    upk = tuple(t[keep] for t in up)
    args = (grids, params, dec_b, sc.bound, ro[keep], rd[keep], "color", dep[keep], upk)
    ref32 = oracle_render_grads(*args)
    ref64 = oracle_render_grads(*args, f64=True)
    scores = score_vs_truth(got, ref32, ref64)
    bad = {k: v for k, v in scores.items() if not v[0] <= v[2]}
    assert not bad, bad


@pytest.mark.gpu
def test_all_rays_dropped():
    """Every ray rejected: zero outputs, zero loss, zero gradients (no NaN from the empty
    batch's max)."""
    sc, grids, params, ro, rd, dep, col, keep = _case(64, seed=44)
    none = torch.zeros_like(keep)
    om, lm, gm = _run(sc, grids, params, ro, rd, dep, col, none, "ba", True)
    assert lm == 0.0
    for k, v in list(om.items()) + list(gm.items()):
        assert torch.isfinite(v).all() and not bool(v.any()), k


@pytest.mark.gpu
def test_non_finite_dropped_rays_stay_out():
    """A dropped ray with a zero direction component and a NaN depth (the reference's filter
    puts NaN on the outside) must not leak non-finite values into any kept output or
    gradient."""
    sc, grids, params, ro, rd, dep, col, keep = _case(128, seed=55)
    ro, rd, dep = ro.clone(), rd.clone(), dep.clone()
    bad = (~keep).nonzero().squeeze(1)[:4]
    rd[bad[0]] = torch.tensor([0.0, 0.0, 0.0])
    dep[bad[1]] = float("nan")
    ro[bad[2]] = torch.tensor([float("inf"), 0.0, 0.0])
    rd[bad[3], 0] = 0.0
    om, lm, gm = _run(sc, grids, params, ro, rd, dep, col, keep, "ba", True)
    oc, lc, gc = _run(sc, grids, params, ro[keep], rd[keep], dep[keep], col[keep], None, "ba", True)
    assert abs(lm - lc) <= 1e-6 * max(abs(lc), 1.0)
    for k in ("depth", "var", "color"):
        assert torch.equal(om[k][keep], oc[k]), k
    for k in gm:
        assert torch.isfinite(gm[k]).all(), k
        if not k.startswith("grad/rays"):
            assert rel_err(gm[k], gc[k]) <= 1e-6, k


@pytest.mark.gpu
def test_masked_step_graph_replay_follows_the_mask():
    """render_batch_loss with ray_mask captured once (nicecore.graph.GraphedStep), the mask
    buffer rewritten in place between replays: each replay equals the eager masked step."""
    from nicecore.graph import GraphedStep
    sc, grids, params, ro, rd, dep, col, keep = _case(256, seed=66)
    model, g, ro_g, rd_g = _leaves(sc, grids, params, ro, rd, "ba")
    r = make_renderer(sc.bound)
    gt, gtc = dep.cuda(), col.cuda()
    mask = keep.cuda().clone()
    leaves = [g[k] for k in ("grid_middle", "grid_fine", "grid_color")] + \
        [p for n, p in model.named_parameters() if not n.startswith("coarse_decoder.")] + [ro_g, rd_g]

    def body():
        for t in leaves:
            t.grad = None
        d, u, c, loss = r.render_batch_loss(g, model, rd_g, ro_g, "cuda", "color", gt, gtc, loss="mapper",
                                            w_color_loss=0.2, color_term=True, ray_mask=mask)
        loss.backward()
        return loss.detach()

    masks = [keep, torch.roll(keep, 7), torch.ones_like(keep)]
    eager = []
    for mk in masks:
        mask.copy_(mk.cuda())
        lv = body()
        eager.append((float(lv), [t.grad.detach().clone() for t in leaves]))
    step = GraphedStep(body)
    for (l0, g0), mk in zip(eager, masks):
        mask.copy_(mk.cuda())
        loss = step()
        torch.cuda.synchronize()
        assert abs(float(loss) - l0) <= 1e-6 * max(abs(l0), 1.0)
        for t, gr in zip(leaves, g0):
            assert rel_err(t.grad.cpu(), gr.cpu()) <= 1e-6
