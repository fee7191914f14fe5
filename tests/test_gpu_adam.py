"""The Mapper's optimiser step on the device (nc_adam_step, nicecore.optim; ABI v7).

Oracles are PyTorch's own optimisers on the same device (the reference constructs
torch.optim.Adam, src/Mapper.py:462-485, and steps it at :625):
  * nicecore.optim.Adam vs torch.optim.Adam(fused=True), whose arithmetic k_adam_dense
    restates (ATen fused_adam_utils.cuh, with its moment updates contracted to
    fma(beta, moment, (1 - beta) * grad) in double as the fused kernel is compiled):
    bit-identical (ADAM_ULPS = 0) over several steps, weight decay and per-group lr
    included, for flat parameters, odd sizes (scalar tail), misaligned views and
    channels-last grids;
  * the same vs the default (foreach) torch.optim.Adam: 1e-6 relative (different
    rounding order);
  * SparseGridAdam vs torch.optim.SparseAdam on the channels-last row view with
    SparseGridGrads.coo() as the gradient (torch/optim/_functional.py sparse_adam,
    all float32 elementwise): bit-identical; untouched voxels unchanged; NCDHW grids;
  * one Mapper iteration: render + loss + backward through the core, then the step,
    matches torch's fused Adam on the same gradients.
"""
import pytest
import torch

ADAM_ULPS = 0


def _ulps(a, b):
    ia = a.detach().float().contiguous().view(torch.int32).long()
    ib = b.detach().float().contiguous().view(torch.int32).long()
    ia = torch.where(ia < 0, -(ia & 0x7FFFFFFF), ia)
    ib = torch.where(ib < 0, -(ib & 0x7FFFFFFF), ib)
    return int((ia - ib).abs().max()) if a.numel() else 0


def _params(seed):
    g = torch.Generator().manual_seed(seed)
    shapes = [(1000,), (1001,), (33, 3), (7,)]
    ps = [torch.randn(s, generator=g).cuda() for s in shapes]
    grid = torch.randn(1, 32, 5, 6, 7, generator=g).cuda().contiguous(memory_format=torch.channels_last_3d)
    base = torch.randn(1 + 4099, generator=g).cuda()
    ps += [grid, base[1:]]  # base[1:] is 4 B past a 16-B boundary: the scalar path
    return ps


def _grads(ps, seed):
    g = torch.Generator().manual_seed(seed)
    return [(torch.randn(p.shape, generator=g) * 10 ** torch.randint(-4, 2, (1,), generator=g)).cuda()
            .to(memory_format=torch.channels_last_3d if p.dim() == 5 else torch.contiguous_format) for p in ps]


def _run(opt_cls, ps, steps, wd, **kw):
    mine = [torch.nn.Parameter(p.clone()) for p in ps]
    groups = [{"params": mine[:3], "lr": 1e-2}, {"params": mine[3:], "lr": 3e-3, "weight_decay": wd}]
    opt = opt_cls(groups, betas=(0.9, 0.999), eps=1e-8, **kw)
    for s in range(steps):
        for p, g in zip(mine, _grads(ps, 100 + s)):
            p.grad = g
        opt.step()
    torch.cuda.synchronize()
    return mine, opt


@pytest.mark.gpu
@pytest.mark.parametrize("wd", [0.0, 1e-2])
def test_adam_matches_torch_fused(wd):
    from nicecore.optim import Adam
    ps = _params(1)
    got, opt = _run(Adam, ps, 5, wd)
    ref, ropt = _run(torch.optim.Adam, ps, 5, wd, fused=True)
    worst = 0
    for a, b in zip(got, ref):
        assert a.stride() == b.stride()
        worst = max(worst, _ulps(a, b))
    for a, b in zip(got, ref):
        sa, sb = opt.state[a], ropt.state[b]
        worst = max(worst, _ulps(sa["exp_avg"], sb["exp_avg"]), _ulps(sa["exp_avg_sq"], sb["exp_avg_sq"]))
        assert float(sa["step"]) == float(sb["step"]) == 5.0
    print(f"max ulp difference vs fused torch.optim.Adam: {worst}")
    assert worst <= ADAM_ULPS


@pytest.mark.gpu
def test_adam_matches_torch_default():
    from nicecore.optim import Adam
    ps = _params(2)
    got, _ = _run(Adam, ps, 4, 1e-3)
    ref, _ = _run(torch.optim.Adam, ps, 4, 1e-3)
    for a, b in zip(got, ref):
        assert torch.allclose(a, b, rtol=1e-6, atol=1e-7)


@pytest.mark.gpu
def test_adam_state_dict_and_scheduler():
    """StepLR (Mapper.py:485) and state_dict round trips work as with torch.optim.Adam."""
    from nicecore.optim import Adam
    ps = _params(3)
    got, opt = _run(Adam, ps, 2, 0.0)
    sched = torch.optim.lr_scheduler.StepLR(opt, step_size=1, gamma=0.5)
    sched.step()
    assert opt.param_groups[0]["lr"] == pytest.approx(5e-3)
    sd = opt.state_dict()
    opt2 = Adam([{"params": got[:3], "lr": 1}, {"params": got[3:], "lr": 1}])
    opt2.load_state_dict(sd)
    assert float(opt2.state[got[0]]["step"]) == 2.0
    assert torch.equal(opt2.state[got[4]]["exp_avg"], opt.state[got[4]]["exp_avg"])


@pytest.mark.gpu
def test_adam_refuses_cpu_and_mixed_strides():
    from nicecore import _lib as L
    from nicecore.optim import adam_step_
    p = torch.zeros(8)
    with pytest.raises(L.NiceCoreError):
        adam_step_(p, p, p, p, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0, step=1)
    q = torch.zeros(4, 4, device="cuda")
    with pytest.raises(L.NiceCoreError):
        adam_step_(q, q.t(), q, q, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0, step=1)


def _synthetic_rows(grid, n, seed):
    """A SparseGridGrads whose rows are set by hand: n random distinct voxels."""
    from nicecore.sparse import SparseGridGrads
    sp = SparseGridGrads({"grid_fine": grid}, keys=("grid_fine",), capacity=n + 5)
    r = sp.rows["grid_fine"]
    g = torch.Generator().manual_seed(seed)
    vox = torch.randperm(r.n_voxels, generator=g)[:n]
    r.row_voxel[:n].copy_(vox)
    r.values[:n].copy_(torch.randn(n, 32, generator=g))
    r.values[n:].fill_(float("nan"))  # beyond the count: never read
    r.count.fill_(n)
    return sp


def _row_view(grid):
    """[D*H*W, 32] view, row = voxel (z*H + y)*W + x."""
    return grid.permute(0, 2, 3, 4, 1).reshape(-1, 32) if grid.is_contiguous(
        memory_format=torch.channels_last_3d) else grid.reshape(32, -1).t()


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["channels_last", "ncdhw"])
def test_sparse_grid_adam_matches_torch_sparse_adam(layout):
    from nicecore.optim import SparseGridAdam
    gen = torch.Generator().manual_seed(9)
    grid = torch.randn(1, 32, 6, 7, 9, generator=gen).cuda()
    if layout == "channels_last":
        grid = grid.contiguous(memory_format=torch.channels_last_3d)
    grid0 = grid.clone()
    ref = torch.nn.Parameter(_row_view(grid).clone())
    ropt = torch.optim.SparseAdam([ref], lr=1e-2, betas=(0.9, 0.999), eps=1e-8)
    opt = None
    touched = torch.zeros(ref.shape[0], dtype=torch.bool, device="cuda")
    for s, n in enumerate([50, 120, 0, 77]):
        sp = _synthetic_rows(grid, n, seed=s)
        if opt is None:
            opt = SparseGridAdam({"grid_fine": grid}, sp, lr=1e-2)
        opt.sparse = sp
        opt.step()
        ref.grad = sp.coo("grid_fine")
        ropt.step()
        touched[sp.indices("grid_fine")] = True
    torch.cuda.synchronize()
    got = _row_view(grid)
    assert torch.equal(got, ref.detach())
    assert torch.equal(got[~touched], _row_view(grid0)[~touched])
    st = ropt.state[ref]
    assert torch.equal(_row_view(opt.state["grid_fine"]["exp_avg"]), st["exp_avg"])
    assert torch.equal(_row_view(opt.state["grid_fine"]["exp_avg_sq"]), st["exp_avg_sq"])


@pytest.mark.gpu
def test_sparse_grid_adam_after_render():
    """C5 flow on room0: sparse rows from a render + backward, then SparseGridAdam ==
    torch.optim.SparseAdam with coo()."""
    from nicecore.optim import SparseGridAdam
    from nicecore.sparse import SparseGridGrads
    from test_gpu_sparse import _run as render, _setup
    sc, g, model, ro, rd, dep = _setup(400, seed=81)
    sp = SparseGridGrads(g, keys=("grid_fine", "grid_color"))
    render(sc, g, model, ro, rd, dep, sparse=sp)
    refs = {k: torch.nn.Parameter(_row_view(g[k]).detach().clone()) for k in sp.rows}
    with torch.no_grad():
        SparseGridAdam(g, sp, lr=5e-3).step()
    for k, p in refs.items():
        p.grad = sp.coo(k)
        torch.optim.SparseAdam([p], lr=5e-3).step()
        assert torch.equal(_row_view(g[k]).detach(), p.detach()), k


@pytest.mark.gpu
def test_mapper_iteration_step():
    """render_batch_loss + backward through the core, then nicecore.optim.Adam with the
    Mapper's param groups vs torch.optim.Adam(fused=True) on the same gradients."""
    from nicecore.optim import Adam
    from test_gpu_loss import _setup as loss_setup
    rec, stage, model, g, ro, rd, r = loss_setup("color_depth", want_rays=False)
    gt, gtc = rec["gt_depth"].cuda(), rec["gt_color"].cuda()
    d, v, c, L = r.render_batch_loss(g, model, rd, ro, "cuda", stage, gt, gtc, loss="mapper", color_term=True)
    L.backward()
    dec = [p for p in model.color_decoder.parameters() if p.grad is not None]
    grids = [g[k] for k in ("grid_middle", "grid_fine", "grid_color")]
    clones = [torch.nn.Parameter(t.detach().clone()) for t in dec + grids]
    for cl, t in zip(clones, dec + grids):
        cl.grad = t.grad.clone()

    def groups(ts):
        return [{"params": ts[:len(dec)], "lr": 1e-3}, {"params": ts[len(dec):len(dec) + 1], "lr": 0.0},
                {"params": ts[len(dec) + 1:], "lr": 5e-3}]
    Adam(groups(dec + grids)).step()
    torch.optim.Adam(groups(clones), fused=True).step()
    torch.cuda.synchronize()
    for a, b in zip(dec + grids, clones):
        assert _ulps(a, b) <= ADAM_ULPS


@pytest.mark.gpu
def test_sharded_sparse_adam_two_gloo_ranks(tmp_path):
    """ZeRO-style ShardedSparseGridAdam over two gloo ranks on one GPU
    (subprocesses, tests/zero_adam_worker.py): bit-identical to the unsharded
    allreduce + SparseGridAdam on every rank, and the replicas agree."""
    import os
    import subprocess
    import sys
    from conftest import REPO
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29637", HSA_ENABLE_IPC_MODE_LEGACY="0")
    procs = [subprocess.Popen([sys.executable, os.path.join(REPO, "tests", "zero_adam_worker.py"), str(tmp_path)],
                              env=dict(env, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r))) for r in range(2)]
    for p in procs:
        assert p.wait(timeout=110) == 0
    outs = [torch.load(tmp_path / f"zero_rank{r}.pt", weights_only=True) for r in range(2)]
    assert set(outs[0]) == set(outs[1])
    for k in outs[0]:
        assert torch.equal(outs[0][k], outs[1][k]), k
    assert outs[0]["grid_fine/1/idx"].numel() > 0


@pytest.mark.gpu
def test_adam_many_parameters_one_call():
    """More parameters than one k_adam_multi launch holds (32), mixed sizes including
    empty and single-element ones, three param groups: still bit-identical to fused Adam."""
    from nicecore.optim import Adam
    g = torch.Generator().manual_seed(11)
    sizes = [int(s) for s in torch.randint(0, 3000, (37,), generator=g)] + [1, 0, 4096 * 64 + 3]
    ps = [torch.randn(s, generator=g).cuda() for s in sizes]

    def run(cls, **kw):
        mine = [torch.nn.Parameter(p.clone()) for p in ps]
        groups = [{"params": mine[:10], "lr": 1e-2}, {"params": mine[10:30], "lr": 0.0},
                  {"params": mine[30:], "lr": 2e-3, "weight_decay": 1e-2}]
        opt = cls(groups, **kw)
        for s in range(3):
            gg = torch.Generator().manual_seed(50 + s)
            for p in mine:
                p.grad = torch.randn(p.shape, generator=gg).cuda()
            opt.step()
        torch.cuda.synchronize()
        return mine, opt
    got, opt = run(Adam)
    ref, ropt = run(torch.optim.Adam, fused=True)
    for a, b in zip(got, ref):
        assert torch.equal(a, b)
        assert torch.equal(opt.state[a]["exp_avg_sq"], ropt.state[b]["exp_avg_sq"])


@pytest.mark.gpu
def test_adam_capturable_matches_torch_fused():
    """capturable=True: step counts on the device, incremented by the launch; same
    arithmetic as torch's fused Adam (which also reads a float32 device step)."""
    from nicecore.optim import Adam
    ps = _params(5)
    got, opt = _run(Adam, ps, 4, 1e-2, capturable=True)
    ref, ropt = _run(torch.optim.Adam, ps, 4, 1e-2, fused=True)
    for a, b in zip(got, ref):
        assert torch.equal(a, b)
        assert opt.state[a]["step"].device.type == "cuda" and float(opt.state[a]["step"]) == 4.0


@pytest.mark.gpu
def test_mapper_iteration_in_one_graph():
    """render + loss + backward + Adam step captured in ONE hipGraph (capturable Adam)
    and replayed: the same parameters as running the iteration eagerly as many times.
    Decoder-only gradients (no float atomics on their path): bit-identical."""
    from nicecore.graph import GraphedStep
    from nicecore.optim import Adam
    from test_gpu_loss import _setup as loss_setup

    def make():
        rec, stage, model, g, ro, rd, r = loss_setup("color_depth", want_rays=False)
        for v in g.values():
            v.requires_grad_(False)
        dec = list(model.color_decoder.parameters())
        for p in model.parameters():
            p.requires_grad_(False)
        for p in dec:
            p.requires_grad_(True)
        opt = Adam([{"params": dec, "lr": 5e-3}], capturable=True)
        gt, gtc = rec["gt_depth"].cuda(), rec["gt_color"].cuda()

        def body():
            for p in dec:
                p.grad = None
            d, u, c, L = r.render_batch_loss(g, model, rd, ro, "cuda", stage, gt, gtc, loss="mapper",
                                             color_term=True)
            L.backward()
            opt.step()
            return L
        return dec, body

    dec_e, body_e = make()
    for _ in range(3 + 4):
        body_e()
    dec_g, body_g = make()
    step = GraphedStep(body_g, warmup=3)  # the warmup runs 3 eager iterations
    for _ in range(4):
        step()
    torch.cuda.synchronize()
    for a, b in zip(dec_g, dec_e):
        assert torch.equal(a, b)
