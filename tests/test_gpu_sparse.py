"""Sparse (touched-voxel) grid gradients, nc_grid.grad_rows (ABI v5).

The reference's grid gradient is dense (autograd grid.grad; Mapper.py:392-404,
:620-627).  nicecore.sparse.SparseGridGrads keeps only the rows of the voxels a batch
touched.  Checks, on the Replica room0 geometry:
  * the rows, scattered back to a dense tensor, equal the dense path's gradient
    (float atomics: 1e-5 of max-abs; NC_DETERMINISTIC: bit-identical), and every
    voxel with a non-zero dense gradient has a row;
  * rays / decoder gradients are unchanged by the mode;
  * claims accumulate over several forwards before one backward, and zero_grad
    restores an all -1 map;
  * the multi-rank merge (nc_sparse_rows_merge) gives every rank the same ascending
    union, and the sum of the ranks' permuted rows is the full batch's gradient --
    in one process over two ray shards, and over two gloo ranks (subprocesses).
"""
import os
import subprocess
import sys

import pytest
import torch

from conftest import REPO
from parity_common import build_model, rel_err
from test_gpu_parity import _room0_case

KEYS = ("grid_middle", "grid_fine", "grid_color")


def _setup(n_rays, stage="color", seed=31):
    sc, grids, params, ro, rd, dep = _room0_case(n_rays, stage, seed=seed)
    model = build_model(params, sc.bound, sc.bound * 2, "cuda")
    g = {k: v.cuda().contiguous(memory_format=torch.channels_last_3d).requires_grad_(True)
         for k, v in grids.items()}
    return sc, g, model, ro.cuda(), rd.cuda(), dep.cuda()


def _run(sc, g, model, ro, rd, dep, sparse=None, deterministic=None, stage="color", dmax=None):
    from nicecore.ops import render_rays
    ro_ = ro.clone().requires_grad_(True)
    rd_ = rd.clone().requires_grad_(True)
    d, u, c = render_rays(model, g, ro_, rd_, sc.bound, stage, dep, depth_max=dmax,
                          deterministic=deterministic, sparse_grads=sparse)
    gen = torch.Generator().manual_seed(5)
    up = [torch.randn(d.shape, generator=gen, dtype=torch.float64).cuda(),
          torch.randn(u.shape, generator=gen, dtype=torch.float64).cuda(),
          torch.randn(c.shape, generator=gen).cuda()]
    torch.autograd.backward([d, u, c], up)
    return ro_.grad, rd_.grad


def _clear(g, model):
    for v in g.values():
        v.grad = None
    for p in model.parameters():
        p.grad = None


@pytest.mark.gpu
@pytest.mark.parametrize("deterministic", [False, True])
def test_sparse_rows_equal_dense_gradient(deterministic):
    from nicecore.sparse import SparseGridGrads
    sc, g, model, ro, rd, dep = _setup(700)
    gro_d, grd_d = _run(sc, g, model, ro, rd, dep, deterministic=deterministic)
    dense = {k: g[k].grad.detach().clone() for k in KEYS}
    pgrad = {n: p.grad.detach().clone() for n, p in model.named_parameters() if p.grad is not None}
    _clear(g, model)
    sp = SparseGridGrads(g, capacity=1024)  # grows on the first forward
    gro_s, grd_s = _run(sc, g, model, ro, rd, dep, sparse=sp, deterministic=deterministic)
    for k in KEYS:
        assert g[k].grad is None, k  # no dense gradient in sparse mode
        n = sp.count(k)
        idx = sp.indices(k)
        assert 0 < n <= 8 * 700 * 48
        assert torch.unique(idx).numel() == n  # one row per voxel
        got = sp.to_dense(k)
        if deterministic:
            assert torch.equal(got, dense[k]), k
        else:
            assert rel_err(got, dense[k]) <= 1e-5, (k, rel_err(got, dense[k]))
        nz = dense[k].permute(0, 2, 3, 4, 1).reshape(-1, 32).abs().amax(1) > 0
        has = torch.zeros_like(nz)
        has[idx] = True
        assert bool((has | ~nz).all()), k  # every voxel with a gradient has a row
        coo = sp.coo(k)
        assert coo.shape == (nz.numel(), 32)
    assert torch.equal(gro_s, gro_d) or rel_err(gro_s, gro_d) <= 1e-6
    assert rel_err(grd_s, grd_d) <= 1e-6
    for n, p in model.named_parameters():
        if n in pgrad:
            assert rel_err(p.grad, pgrad[n]) <= 1e-5, n
    sp.zero_grad()
    for k in KEYS:
        assert sp.count(k) == 0
        assert bool((sp.rows[k].map == -1).all()), k


@pytest.mark.gpu
@pytest.mark.parametrize("deterministic", [False, True])
def test_sparse_rows_accumulate_over_forwards(deterministic):
    """Two renders, one backward (claims accumulate until zero_grad); then a second
    step after zero_grad sees only its own batch.  NC_DETERMINISTIC adds each voxel
    run to its row (nc_det.hip det_add), so the second backward keeps the first's rows."""
    from nicecore.ops import render_rays
    from nicecore.sparse import SparseGridGrads
    sc, g, model, ro, rd, dep = _setup(600, seed=41)
    dmax = dep.max().reshape(1)
    a, b = slice(0, 300), slice(300, 600)
    ref = {}
    for sl in (a, b):
        _run(sc, g, model, ro[sl], rd[sl], dep[sl], dmax=dmax, deterministic=deterministic)
        for k in KEYS:
            ref[k] = ref.get(k, 0) + g[k].grad.detach().clone()
        _clear(g, model)
    sp = SparseGridGrads(g)
    outs = []
    gen = torch.Generator().manual_seed(5)
    for sl in (a, b):
        d, u, c = render_rays(model, g, ro[sl], rd[sl], sc.bound, "color", dep[sl], depth_max=dmax,
                              sparse_grads=sp, deterministic=deterministic)
        gen = torch.Generator().manual_seed(5)  # same upstream as _run per shard
        up = [torch.randn(d.shape, generator=gen, dtype=torch.float64).cuda(),
              torch.randn(u.shape, generator=gen, dtype=torch.float64).cuda(),
              torch.randn(c.shape, generator=gen).cuda()]
        outs.append(((d * up[0]).sum() + (u * up[1]).sum() + (c * up[2]).sum().double()))
    (outs[0] + outs[1]).backward()
    for k in KEYS:
        if deterministic:  # two fp32 sums of the same two bit-identical per-batch rows
            assert torch.equal(sp.to_dense(k), ref[k]), k
        else:
            assert rel_err(sp.to_dense(k), ref[k]) <= 1e-5, k
    sp.zero_grad()
    _clear(g, model)
    _run(sc, g, model, ro[a], rd[a], dep[a], dmax=dmax, deterministic=deterministic)
    only_a = {k: g[k].grad.detach().clone() for k in KEYS}
    _clear(g, model)
    _run(sc, g, model, ro[a], rd[a], dep[a], sparse=sp, dmax=dmax, deterministic=deterministic)
    for k in KEYS:
        if deterministic:
            assert torch.equal(sp.to_dense(k), only_a[k]), k
        else:
            assert rel_err(sp.to_dense(k), only_a[k]) <= 1e-5, k


@pytest.mark.gpu
def test_sparse_rows_eval_points():
    """NICE.forward on caller points (nc_points_*) with sparse grid rows."""
    from nicecore.ops import eval_points
    from nicecore.sparse import SparseGridGrads
    sc, g, model, ro, rd, dep = _setup(10, seed=43)
    gen = torch.Generator().manual_seed(3)
    lo, hi = sc.bound[:, 0], sc.bound[:, 1]
    p = (lo + (hi - lo) * torch.rand(5000, 3, generator=gen, dtype=torch.float64)).float().cuda()
    up = torch.randn(5000, 4, generator=gen).cuda()
    (eval_points(model, p, g, "color") * up).sum().backward()
    dense = {k: g[k].grad.detach().clone() for k in KEYS}
    _clear(g, model)
    sp = SparseGridGrads(g)
    (eval_points(model, p, g, "color", sparse_grads=sp) * up).sum().backward()
    for k in KEYS:
        assert rel_err(sp.to_dense(k), dense[k]) <= 1e-5, k


def _merge(sp_in, world_lists, counts, key):
    """nc_sparse_rows_merge of one grid, as SparseGridGrads.allreduce runs it."""
    import ctypes
    from nicecore import _lib as L
    lib = L.load()
    r = sp_in.rows[key]
    cap = world_lists.shape[1]
    world = world_lists.shape[0]
    out_cap = min(world * cap, r.n_voxels)
    vals = torch.empty(out_cap, 32, device="cuda")
    rv = torch.empty(out_cap, dtype=torch.int64, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
    nb = lib.nc_sparse_merge_temp_bytes(world * cap, r.n_voxels)
    tmp = torch.empty(nb, dtype=torch.uint8, device="cuda")
    sin, sout = r.struct(), r.struct(values=vals, row_voxel=rv, count=cnt, capacity=out_cap)
    L.check(lib.nc_sparse_rows_merge(ctypes.byref(sin), ctypes.byref(sout), world_lists.reshape(-1).data_ptr(),
                                     counts.data_ptr(), world, cap, tmp.data_ptr(), nb,
                                     torch.cuda.current_stream().cuda_stream), "merge")
    n = int(cnt.item())
    return rv[:n].clone(), vals[:n].clone()


@pytest.mark.gpu
def test_sparse_merge_two_shards_one_process():
    from nicecore.sparse import SparseGridGrads
    sc, g, model, ro, rd, dep = _setup(800, seed=47)
    dmax = dep.max().reshape(1)
    _run(sc, g, model, ro, rd, dep, dmax=dmax)
    full = {k: g[k].grad.detach().clone() for k in KEYS}
    _clear(g, model)
    shards = [SparseGridGrads(g), SparseGridGrads(g)]
    for s, sl in zip(shards, (slice(0, 400), slice(400, 800))):
        _run(sc, g, model, ro[sl], rd[sl], dep[sl], sparse=s, dmax=dmax)
    # shards' upstream gradients are the first / second halves of _run's randn draws
    # only if drawn per shard: compare against per-shard dense runs instead
    ref = {}
    for sl in (slice(0, 400), slice(400, 800)):
        _clear(g, model)
        _run(sc, g, model, ro[sl], rd[sl], dep[sl], dmax=dmax)
        for k in KEYS:
            ref[k] = ref.get(k, 0) + g[k].grad.detach().clone()
    for k in KEYS:
        cap = max(s.rows[k].capacity for s in shards)
        lists = torch.full((2, cap), -1, dtype=torch.int64, device="cuda")
        counts = torch.empty(2, dtype=torch.int32, device="cuda")
        for i, s in enumerate(shards):
            lists[i, :s.rows[k].capacity] = s.rows[k].row_voxel
            counts[i] = s.rows[k].count[0]
        merged = [_merge(s, lists, counts, k) for s in shards]
        assert torch.equal(merged[0][0], merged[1][0])  # same union, same order on both ranks
        u = merged[0][0]
        assert bool((u[1:] > u[:-1]).all())  # ascending, no duplicates
        both = torch.cat([s.indices(k) for s in shards])
        assert torch.equal(u, torch.unique(both))
        total = merged[0][1] + merged[1][1]
        D, H, W = shards[0].rows[k].shape
        dense = torch.zeros(D * H * W, 32, device="cuda")
        dense[u] = total
        dense = dense.reshape(1, D, H, W, 32).permute(0, 4, 1, 2, 3)
        assert rel_err(dense, ref[k]) <= 1e-5, k
        assert full[k].shape == dense.shape


@pytest.mark.gpu
def test_sparse_allreduce_two_gloo_ranks(tmp_path):
    """SparseGridGrads.allreduce over 2 gloo ranks (subprocesses on this GPU) equals
    the single-process gradient of the whole batch."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29631", HSA_ENABLE_IPC_MODE_LEGACY="0")
    procs = []
    for r in range(2):
        e = dict(env, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, os.path.join(REPO, "tests", "sparse_dist_worker.py"),
                                       str(tmp_path)], env=e))
    for p in procs:
        assert p.wait(timeout=110) == 0
    outs = [torch.load(tmp_path / f"rank{r}.pt", weights_only=True) for r in range(2)]
    sc, g, model, ro, rd, dep = _setup(512, seed=53)
    dmax = dep.max().reshape(1)
    ref = {}
    for sl in (slice(0, 256), slice(256, 512)):
        _clear(g, model)
        _run(sc, g, model, ro[sl], rd[sl], dep[sl], dmax=dmax)
        for k in KEYS:
            ref[k] = ref.get(k, 0) + g[k].grad.detach().clone().cpu()
    for k in KEYS:
        assert torch.equal(outs[0][k + "/idx"], outs[1][k + "/idx"])
        assert torch.equal(outs[0][k + "/val"], outs[1][k + "/val"])  # the all-reduced rows agree
        D, H, W = ref[k].shape[2:]
        dense = torch.zeros(D * H * W, 32)
        dense[outs[0][k + "/idx"]] = outs[0][k + "/val"]
        dense = dense.reshape(1, D, H, W, 32).permute(0, 4, 1, 2, 3)
        assert rel_err(dense, ref[k]) <= 1e-5, k


@pytest.mark.gpu
def test_sparse_rows_drive_sparse_adam():
    """coo() is the gradient of the channels-last row view: a torch.optim.SparseAdam step
    with it equals the SparseAdam step with the dense path's gradient made sparse
    (SparseAdam's eps enters after the bias correction, unlike dense Adam's, so the
    comparison is sparse-with-sparse)."""
    from nicecore.sparse import SparseGridGrads
    sc, g, model, ro, rd, dep = _setup(300, seed=71)
    # ordered reductions: the sparse and dense gradients are bit-identical, so entries
    # whose contributions cancel cannot flip sign between the two
    _run(sc, g, model, ro, rd, dep, deterministic=True)
    dense = g["grid_fine"].grad.detach().permute(0, 2, 3, 4, 1).reshape(-1, 32).clone()
    _clear(g, model)
    sp = SparseGridGrads(g, keys=("grid_fine",))
    _run(sc, g, model, ro, rd, dep, sparse=sp, deterministic=True)
    grid = g["grid_fine"]
    rows = grid.detach().permute(0, 2, 3, 4, 1).reshape(-1, 32)  # a view of the channels-last grid
    assert rows.data_ptr() == grid.data_ptr()
    ps = torch.nn.Parameter(rows.clone())
    ps.grad = sp.coo("grid_fine")
    torch.optim.SparseAdam([ps], lr=1e-2).step()
    pd = torch.nn.Parameter(rows.clone())
    pd.grad = dense.to_sparse(sparse_dim=1)
    torch.optim.SparseAdam([pd], lr=1e-2).step()
    assert torch.allclose(ps.detach(), pd.detach(), rtol=0, atol=1e-7)
    assert not torch.equal(ps.detach(), rows)


@pytest.mark.gpu
def test_sparse_rows_overflow_is_reported():
    """A capacity smaller than the claims (rows fixed by hand, no growth) is reported,
    not silently truncated."""
    from nicecore import _lib as L
    from nicecore.sparse import SparseGridGrads
    sc, g, model, ro, rd, dep = _setup(200, seed=73)
    sp = SparseGridGrads(g, keys=("grid_fine",), capacity=16)
    r = sp.rows["grid_fine"]
    r.reserve = lambda extra: None  # keep the 16 rows
    _run(sc, g, model, ro, rd, dep, sparse=sp)
    with pytest.raises(L.NiceCoreError, match="overflowed"):
        sp.count("grid_fine")
    sp.zero_grad()
    assert bool((r.map == -1).all())
