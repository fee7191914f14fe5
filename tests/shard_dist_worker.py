"""Rank worker of tests/test_gpu_configs.py::test_c4_apartment_two_gloo_ranks_equal_full_batch:
renders its 625-ray half of the 1250-ray Apartment batch with the MAX pre-reduce of the
depth bound (distributed.global_depth_max) and SUM-reduces the grid and decoder
gradients (distributed.allreduce_grads), as bench.py's N > 1 step does; saves the result."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "nice-slam-annotation_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main(out):
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    from test_gpu_configs import shard_collect, shard_setup, shard_step
    from nicecore import distributed as ND
    sc, g, model, ro, rd, dep, col = shard_setup()
    ro, rd, dep, col = ND.shard(rank, world, ro, rd, dep, col)
    dmax = ND.global_depth_max(dep)
    res = shard_step(sc, g, model, ro, rd, dep, col, dmax)
    ND.allreduce_grads(list(g.values()) + list(model.parameters()))
    torch.cuda.synchronize()
    torch.save(shard_collect(res, g, model), os.path.join(out, f"shard_rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
