"""Rank worker of tests/test_gpu_sparse.py::test_sparse_allreduce_two_gloo_ranks:
renders its half of a 512-ray batch with sparse grid gradients, all-reduces them
(SparseGridGrads.allreduce over gloo) and saves the union rows."""
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
    from test_gpu_sparse import KEYS, _run, _setup
    from nicecore.sparse import SparseGridGrads
    sc, g, model, ro, rd, dep = _setup(512, seed=53)
    dmax = dep.max().reshape(1)
    sl = slice(256 * rank, 256 * (rank + 1))
    sp = SparseGridGrads(g)
    _run(sc, g, model, ro[sl], rd[sl], dep[sl], sparse=sp, dmax=dmax)
    sp.allreduce()
    res = {}
    for k in KEYS:
        res[k + "/idx"] = sp.indices(k).cpu()
        res[k + "/val"] = sp.values(k).cpu()
    torch.save(res, os.path.join(out, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
