"""cProfile of bench.py's training step (host side).  Run on a GPU box:
    python tools/host_profile.py [--steps 200]
Prints the host time per step and the top functions by cumulative time."""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import torch  # noqa: E402

if __name__ == "__main__":
    sys.argv = [sys.argv[0]] + [a for a in sys.argv[1:]]
    args = bench.parse()
    world, rank, local = bench.setup_dist(args)
    device = torch.device("cuda", 0)
    from nicecore import _lib as L
    L.load()
    w = bench.build_workload(args, rank, device, world)
    step, _ = bench.make_step(w, args, world, device)  # the eager step (the drop-in path)
    for _ in range(10):
        step()
    torch.cuda.synchronize()
    n = args.steps
    t0 = time.perf_counter()
    for _ in range(n):
        step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"host enqueue {1e3 * (t1 - t0) / n:.4f} ms/step, wall {1e3 * (t2 - t0) / n:.4f} ms/step")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(n):
        step()
    pr.disable()
    torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats("cumulative").print_stats(45)
    pstats.Stats(pr).sort_stats("tottime").print_stats(30)
    # torch.profiler view of the same step: host time per aten op / autograd node
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU]) as prof:
        for _ in range(20):
            step()
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=40))
