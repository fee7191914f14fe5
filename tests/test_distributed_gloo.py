"""Ray-sharded data parallelism (nicecore.distributed) on 2 gloo ranks.

Each rank renders its contiguous shard of the batch with the CPU oracle, using
the all-reduced batch-global depth max, back-propagates the mapper loss and
all-reduces grid + decoder gradients.  The summed gradients and the gathered ray
gradients must equal a single-process render of the whole batch.  Also shows why
the MAX pre-reduce is required: without it outputs change."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import load_case, load_scene


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _render_loss(O, grids, prm, bound, cbound, ro, rd, dep, col, depth_max=None):
    dec_b = {"coarse": cbound, "middle": bound, "fine": bound, "color": bound}
    d, u, c = O.render_batch_ray(grids, prm, dec_b, bound, rd, ro, "color", dep, depth_max=depth_max)
    loss = ((dep.double() - d).abs() * (dep > 0).double()).sum() + 0.2 * (col - c).abs().sum()
    return loss, d


def _worker(rank, world, port, out):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    import conftest  # noqa: F401  (paths)
    from oracle import nice_oracle as O
    from nicecore import distributed as ND
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    bound, cbound, grids, params = load_scene()
    rec = load_case("color_depth")
    ro, rd, dep, col = ND.shard(rank, world, rec["rays_o"], rec["rays_d"], rec["gt_depth"], rec["gt_color"])
    ro = ro.clone().requires_grad_(True)
    rd = rd.clone().requires_grad_(True)
    g = {k: v.clone().requires_grad_(True) for k, v in grids.items()}
    prm = {k: v.clone().requires_grad_(True) for k, v in params.items()}
    dmax = ND.global_depth_max(dep)
    loss, _ = _render_loss(O, g, prm, bound, cbound, ro, rd, dep, col, depth_max=dmax)
    loss.backward()
    ND.allreduce_grads(list(g.values()) + list(prm.values()))
    gro = [torch.zeros(0)] * world
    sizes = [ND.shard_bounds(rec["rays_o"].shape[0], r, world) for r in range(world)]
    gathered = [torch.zeros(b - a, 3) for a, b in sizes]
    dist.all_gather(gathered, ro.grad.contiguous())
    if rank == 0:
        # numpy copies: torch tensors in an mp.Queue share fds that die with this process
        out.put({"grids": {k: v.grad.numpy().copy() for k, v in g.items() if v.grad is not None},
                 "params": {k: v.grad.numpy().copy() for k, v in prm.items() if v.grad is not None},
                 "rays_o": torch.cat(gathered).numpy().copy()})
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_grads_equal_full_batch():
    from oracle import nice_oracle as O
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    bound, cbound, grids, params = load_scene()
    rec = load_case("color_depth")
    ro = rec["rays_o"].clone().requires_grad_(True)
    rd = rec["rays_d"].clone().requires_grad_(True)
    g = {k: v.clone().requires_grad_(True) for k, v in grids.items()}
    prm = {k: v.clone().requires_grad_(True) for k, v in params.items()}
    loss, _ = _render_loss(O, g, prm, bound, cbound, ro, rd, rec["gt_depth"], rec["gt_color"])
    loss.backward()
    for k, v in res["grids"].items():
        torch.testing.assert_close(torch.from_numpy(v), g[k].grad, rtol=1e-5, atol=1e-7)
    for k, v in res["params"].items():
        torch.testing.assert_close(torch.from_numpy(v), prm[k].grad, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(torch.from_numpy(res["rays_o"]), ro.grad, rtol=1e-6, atol=1e-7)


def test_local_depth_max_changes_outputs():
    """Rendering a shard with its LOCAL max(gt_depth) is not the reference result."""
    from oracle import nice_oracle as O
    from nicecore import distributed as ND
    bound, cbound, grids, params = load_scene()
    rec = load_case("color_depth")
    dec_b = {"coarse": cbound, "middle": bound, "fine": bound, "color": bound}
    full, _, _ = O.render_batch_ray(grids, params, dec_b, bound, rec["rays_d"], rec["rays_o"], "color",
                                    rec["gt_depth"])
    ro, rd, dep = ND.shard(1, 2, rec["rays_o"], rec["rays_d"], rec["gt_depth"])
    a, b = ND.shard_bounds(rec["rays_o"].shape[0], 1, 2)
    local, _, _ = O.render_batch_ray(grids, params, dec_b, bound, rd, ro, "color", dep)
    glob, _, _ = O.render_batch_ray(grids, params, dec_b, bound, rd, ro, "color", dep,
                                    depth_max=rec["gt_depth"].max())
    torch.testing.assert_close(glob, full[a:b], rtol=0, atol=0)
    if float(dep.max()) != float(rec["gt_depth"].max()):
        assert float((local - full[a:b]).abs().max()) > 0


def _shared_buffer_worker(rank, world, port, out):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import conftest  # noqa: F401  (paths)
    from nicecore import distributed as ND
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # leaves whose .grad are views of ONE buffer (as render_fn._alloc_grads makes them,
    # grid-like strided view included) plus one ordinary gradient
    buf = torch.arange(40, dtype=torch.float32) * (rank + 1)
    a = torch.zeros(2, 3, requires_grad=True)
    b = torch.zeros(1, 2, 2, 2, 2, requires_grad=True)   # 16 elements
    c = torch.zeros(18, requires_grad=True)
    d = torch.zeros(5, requires_grad=True)
    a.grad = buf[0:6].view(2, 3)
    b.grad = torch.as_strided(buf, (1, 2, 2, 2, 2), (16, 1, 8, 4, 2), 6)
    c.grad = buf[22:40]
    d.grad = torch.full((5,), float(rank + 1))
    whole, rest = ND._shared_bases([a.grad, b.grad, c.grad, d.grad])
    n_whole = len(whole)
    ND.allreduce_grads([a, b, c, d])
    if rank == 0:
        out.put((n_whole, len(rest), buf.numpy().copy(), d.grad.numpy().copy(), a.grad.numpy().copy()))
    dist.barrier()
    dist.destroy_process_group()


def test_allreduce_shared_gradient_buffer():
    """One collective over a buffer the gradients fully cover; values are summed."""
    import numpy as np
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_shared_buffer_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    n_whole, n_rest, buf, dgrad, agrad = q.get(timeout=120)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert n_whole == 1 and n_rest == 1
    np.testing.assert_array_equal(buf, np.arange(40, dtype=np.float32) * 3)   # 1x + 2x
    np.testing.assert_array_equal(dgrad, np.full(5, 3.0, dtype=np.float32))
    np.testing.assert_array_equal(agrad, buf[0:6].reshape(2, 3))


def test_shared_buffer_ranges():
    """Gradients that tile parts of one buffer are reduced as 1-D ranges of it: the
    grid part and the decoder part of the core's buffer separately (bench.py N > 1
    reduces them at different times), a gap splits a range, a non-view stays apart."""
    from nicecore import distributed as ND
    buf = torch.zeros(64)
    grid = torch.as_strided(buf, (1, 4, 2, 2, 2), (32, 1, 16, 8, 4), 0)   # channels-last-like, 32 floats
    p1, p2 = buf[32:40].view(2, 4), buf[40:48]
    p3 = buf[56:64]
    other = torch.ones(3)
    ranges, rest = ND._shared_bases([grid])
    assert [r.numel() for r in ranges] == [32] and rest == []
    assert ranges[0].data_ptr() == buf.data_ptr() and ranges[0].dim() == 1
    ranges, rest = ND._shared_bases([p2, p1, p3, other])
    assert sorted(r.numel() for r in ranges) == [8, 16] and len(rest) == 1


def test_shared_buffer_after_accumulate_grad():
    """The grads AccumulateGrad stores (detached aliases, no ._base) of views of one
    buffer are still found to share it: grouped by storage, one range."""
    from nicecore import distributed as ND
    buf = torch.zeros(20)

    class Fn(torch.autograd.Function):
        @staticmethod
        def forward(ctx, a, b, c):
            return a.sum() + b.sum() + c.sum()

        @staticmethod
        def backward(ctx, g):
            return (torch.as_strided(buf, (1, 2, 2, 1, 2), (8, 1, 4, 2, 2), 0), buf[8:14].view(2, 3),
                    buf[14:20].detach())
    a = torch.zeros(1, 2, 2, 1, 2).contiguous(memory_format=torch.channels_last_3d).requires_grad_(True)
    b = torch.zeros(2, 3, requires_grad=True)
    c = torch.zeros(6, requires_grad=True)
    Fn.apply(a, b, c).backward()
    assert a.grad._base is None and a.grad.data_ptr() == buf.data_ptr()
    ranges, rest = ND._shared_bases([a.grad, b.grad, c.grad])
    assert rest == [] and [r.numel() for r in ranges] == [20] and ranges[0].data_ptr() == buf.data_ptr()


def _rows_worker(rank, world, port, out):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import conftest  # noqa: F401  (paths)
    from nicecore import distributed as ND
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    gen = torch.Generator().manual_seed(rank)
    grads = [torch.randn(1, 32, 3, 4, 5, generator=gen).contiguous(memory_format=torch.channels_last_3d),
             torch.randn(1, 32, 2, 3, 2, generator=gen).contiguous(memory_format=torch.channels_last_3d)]
    before = [g.clone() for g in grads]
    rows = [torch.tensor([0, 7, 8, 59]), torch.tensor([3, 11])]
    finish = ND.allreduce_rows_async(list(zip(grads, rows)))
    finish()
    out.put((rank, [b.numpy().copy() for b in before], [g.numpy().copy() for g in grads]))
    dist.barrier()
    dist.destroy_process_group()


def test_allreduce_rows_frustum():
    """Frustum-compacted exchange (bench.py N > 1): the selected voxel rows of every
    grid are summed over the ranks, the other rows keep each rank's own values."""
    import numpy as np
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rows_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict((r, (b, a)) for r, b, a in (q.get(timeout=120) for _ in range(world)))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    rows = [[0, 7, 8, 59], [3, 11]]
    for gi in range(2):
        tot = res[0][0][gi] + res[1][0][gi]
        for r in range(world):
            before, after = res[r][0][gi], res[r][1][gi]
            flat_b = np.moveaxis(before, 1, -1).reshape(-1, 32)
            flat_a = np.moveaxis(after, 1, -1).reshape(-1, 32)
            flat_t = np.moveaxis(tot, 1, -1).reshape(-1, 32)
            sel = np.zeros(flat_b.shape[0], bool)
            sel[rows[gi]] = True
            np.testing.assert_allclose(flat_a[sel], flat_t[sel], rtol=0, atol=1e-6)
            np.testing.assert_array_equal(flat_a[~sel], flat_b[~sel])
