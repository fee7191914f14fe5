"""Rank worker of tests/test_gpu_adam.py::test_sharded_sparse_adam_two_gloo_ranks: each
rank renders its half of a batch with sparse grid gradients (ordered reduction, so two
renders give identical rows), then steps one copy of the grids with the unsharded
SparseGridGrads.allreduce + SparseGridAdam and another with ShardedSparseGridAdam, two
iterations, and checks they agree bit for bit (parameters, and this rank's moment
slab against the full moments)."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "nice-slam-annotation_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main(out):
    dist.init_process_group("gloo")
    rank = dist.get_rank()
    torch.cuda.set_device(0)
    from test_gpu_sparse import _run, _setup
    from nicecore.optim import ShardedSparseGridAdam, SparseGridAdam
    from nicecore.sparse import SparseGridGrads
    keys = ("grid_fine", "grid_color")
    sc, g, model, ro, rd, dep = _setup(512, seed=57)
    dmax = dep.max().reshape(1)
    sl = slice(256 * rank, 256 * (rank + 1))
    gA = {k: g[k].detach().clone() for k in keys}
    gB = {k: g[k].detach().clone() for k in keys}
    spA, spB = SparseGridGrads(g, keys=keys), SparseGridGrads(g, keys=keys)
    optA = SparseGridAdam(gA, spA, lr=1e-2)
    optB = ShardedSparseGridAdam(gB, spB, lr=1e-2)
    res = {}
    for it in range(2):
        for sp in (spA, spB):
            sp.zero_grad()
            _run(sc, g, model, ro[sl], rd[sl], dep[sl], sparse=sp, dmax=dmax, deterministic=True)
            for k in keys:
                g[k].grad = None
        spA.allreduce()
        optA.step()
        optB.step()
        torch.cuda.synchronize()
        for k in keys:
            assert torch.equal(gA[k], gB[k]), (it, k)
            v0, v1 = optB.state[k]["slab"]
            for m in ("exp_avg", "exp_avg_sq"):
                full = optA.state[k][m].permute(0, 2, 3, 4, 1).reshape(-1, 32)
                assert torch.equal(full[v0:v1], optB.state[k][m]), (it, k, m)
            idx = spA.indices(k)
            res[f"{k}/{it}/idx"] = idx.cpu()
            res[f"{k}/{it}/rows"] = gB[k].permute(0, 2, 3, 4, 1).reshape(-1, 32)[idx].cpu()
    torch.save(res, os.path.join(out, f"zero_rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
