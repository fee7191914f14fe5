"""The Mapper's unmodified call sequence at bench.py's C2 workload, timed beside the
fused and the graph-replayed steps (what a caller that keeps the
reference's Python loss gets).

    ref        Renderer.render_batch_ray + the reference's loss expression with its boolean
               masks (Mapper.py:598-612) + loss.backward()
    loss_only  ref's loss statement + backward over precomputed render outputs: the
               caller's own share of ref (a render that cost nothing)
    fused      Renderer.render_batch_loss + backward (bench.py's eager step)
    graph      the fused step replayed from a hipGraph (bench.py's value)

Run on a GPU box:  python tools/bench_callseq.py [--steps 200] [--profile]"""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import torch  # noqa: E402


def main():
    prof = "--profile" in sys.argv
    sys.argv = [a for a in sys.argv if a != "--profile"]
    args = bench.parse()
    world, rank, local = bench.setup_dist(args)
    device = torch.device("cuda", 0)
    from nicecore import _lib as L
    from nicecore.graph import GraphedStep
    L.load()
    w = bench.build_workload(args, rank, device, world)
    grids, model, r = w["grids"], w["model"], w["renderer"]
    ro, rd, gt, gtc = w["ro"], w["rd"], w["gt"], w["gtc"]
    leaves = [p for p in model.parameters() if p.requires_grad] + [g for g in grids.values() if g.requires_grad]
    leaves += [ro, rd]
    stage = args.stage
    w_color = 0.2

    def ref():
        for t in leaves:
            t.grad = None
        depth, unc, color = r.render_batch_ray(grids, model, rd, ro, device, stage, gt)
        depth_mask = gt > 0
        loss = torch.abs(gt[depth_mask] - depth[depth_mask]).sum()
        if stage == "color":
            loss += w_color * torch.abs(gtc - color).sum()
        loss.backward()
        return loss

    def fused():
        for t in leaves:
            t.grad = None
        d, u, c, loss = r.render_batch_loss(grids, model, rd, ro, device, stage, gt, gtc, loss="mapper",
                                            w_color_loss=w_color, color_term=stage == "color")
        loss.backward()
        return loss

    # the two statements agree (loss to float rounding, gradients to the float atomics)
    la = float(ref())
    ga = [t.grad.clone() if t.grad is not None else None for t in leaves]
    lb = float(fused())
    gb = [t.grad.clone() if t.grad is not None else None for t in leaves]
    assert [a is None for a in ga] == [b is None for b in gb]
    err = max(float((a - b).abs().max()) / max(float(b.abs().max()), 1e-30)
              for a, b in zip(ga, gb) if a is not None)
    print(f"ref loss {la:.9e} fused loss {lb:.9e} rel {abs(la - lb) / abs(lb):.2e}; max grad rel err {err:.2e}")

    # the caller's own part of ref(): the same loss statement and backward over
    # precomputed render outputs (leaves), i.e. ref() with a render that costs nothing
    d0, u0, c0 = (t.detach() for t in r.render_batch_ray(grids, model, rd, ro, device, stage, gt))
    dl, cl = d0.clone().requires_grad_(True), c0.clone().requires_grad_(True)

    def loss_only():
        dl.grad = cl.grad = None
        depth_mask = gt > 0
        loss = torch.abs(gt[depth_mask] - dl[depth_mask]).sum()
        if stage == "color":
            loss += w_color * torch.abs(gtc - cl).sum()
        loss.backward()
        return loss

    graph = GraphedStep(fused)
    res = {}
    for name, fn in (("ref", ref), ("fused", fused), ("graph", graph), ("ref", ref), ("loss_only", loss_only)):
        for _ in range(args.warmup + 5):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            fn()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        res[name] = (1e3 * (t2 - t0) / args.steps, 1e3 * (t1 - t0) / args.steps)
        print(f"{name:9s} wall {res[name][0]:.4f} ms/step  host enqueue {res[name][1]:.4f} ms/step", flush=True)
    if prof:
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(args.steps):
            ref()
        pr.disable()
        torch.cuda.synchronize()
        pstats.Stats(pr).sort_stats("tottime").print_stats(30)


if __name__ == "__main__":
    main()
