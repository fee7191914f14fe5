"""A whole Tracker iteration on the drop-ins (SURVEY.md §8f rank 2 with the render path):
Tracker.optimize_cam_in_batch (src/Tracker.py:78-135) for Replica room0 — camera tensor
(quaternion + translation, common.py:163-176) -> c2w, 200 pixels sampled on the device
from a resident depth / colour frame (nicecore.sampling.sample_frames: rays, gt and the
bbox pre-filter mask in one launch, Tracker.py:98-111), the boolean compaction of the
reference (one host sync for the count), render_batch_ray + the tracker loss
(handle_dynamic, colour term, w_color_loss 0.5; Tracker.py:113-130) fused in the core,
backward to the camera tensor (the pose-gradient launch), Adam step, loss.item().

Prints one JSON line: ms per iteration (eager, as the unmodified Tracker loop runs it)
and the render + loss + backward share of it (the same rays, timed alone).

    python tools/bench_tracker_iteration.py [--iters 200]
"""
import argparse
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "nice-slam-annotation_amd")]


def camera_from_tensor(q):
    """[qw, qx, qy, qz, tx, ty, tz] -> [3, 4] c2w (unit quaternion rotation | t),
    the convention of common.py:163-176."""
    w, x, y, z = q[0], q[1], q[2], q[3]
    R = torch.stack([
        torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)]),
        torch.stack([2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)]),
        torch.stack([2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]),
    ])
    return torch.cat([R, q[4:7].reshape(3, 1)], dim=1)


def graph_variant(args, r, grids, model, cam, sc, depth_d, color_d, bound, dev):
    """The same iteration replayed as one hipGraph (nicecore.graph.GraphedStep, Adam
    capturable) with the loss read back once per iteration.  There is no compaction, so
    it is timed only when every ray passes the pre-filter (checked)."""
    from nicecore.graph import GraphedStep
    from nicecore.sampling import sample_frames
    E, H, W = args.edge, sc.H, sc.W
    cam_g = cam.detach().clone().requires_grad_(True)
    opt_g = torch.optim.Adam([cam_g], lr=1e-3, capturable=True)

    def body():
        cam_g.grad = None
        c2w = camera_from_tensor(cam_g)
        ro, rd, gd, gc, inside = sample_frames(E, H - E, E, W - E, args.pixels, sc.fx, sc.fy, sc.cx, sc.cy,
                                               c2w.unsqueeze(0), depth_d, color_d, bound=bound, device=dev)
        d, u, c, loss = r.render_batch_loss(grids, model, rd, ro, dev, "color", gd, gc, loss="tracker",
                                            color_term=True, w_color_loss=0.5, handle_dynamic=True)
        loss.backward()
        opt_g.step()
        return loss, inside
    step = GraphedStep(body)
    _, inside = step()
    if not bool(inside.all()):
        return {"graph_error": "a ray failed the bbox pre-filter: the graph variant would skip a compaction"}
    for _ in range(args.warmup):
        step()[0].item()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(args.iters):
        lg = step()[0].item()  # the Tracker's loss.item() sync, once per iteration
    torch.cuda.synchronize()
    g_ms = (time.perf_counter() - t) / args.iters * 1e3
    return {"graph_ms_per_iteration": round(g_ms, 4), "graph_last_loss": lg}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--pixels", type=int, default=200)
    ap.add_argument("--edge", type=int, default=100)
    ap.add_argument("--scene", default="replica_room0")
    ap.add_argument("--graph", action="store_true",
                    help="also replay the iteration as one hipGraph (no compaction: this workload's "
                         "rays all pass the pre-filter, which is checked)")
    args = ap.parse_args()
    import bench
    from nicecore.sampling import sample_frames, bbox_filter
    ns = argparse.Namespace(scene=args.scene, layout="channels_last", rays=16, mode="tracker",
                            sparse_grads="off", fix_fine=False, frustum="off")
    w = bench.build_workload(ns, 0, "cuda")
    sc, r = w["sc"], w["renderer"]
    grids = {k: v.detach() for k, v in w["grids"].items()}
    model = w["model"]
    for p in model.parameters():
        p.requires_grad_(False)
    dev = "cuda"
    # one resident frame: depth within the bound (5 % holes), random colour
    gen = torch.Generator().manual_seed(0)
    depth = torch.rand(sc.H, sc.W, generator=gen) * 2.5 + 0.5
    depth[torch.rand(sc.H, sc.W, generator=gen) < 0.05] = 0.0
    color = torch.rand(sc.H, sc.W, 3, generator=gen)
    depth_d, color_d = depth.cuda().reshape(1, sc.H, sc.W), color.cuda().reshape(1, sc.H, sc.W, 3)
    centre = ((sc.bound[:, 0] + sc.bound[:, 1]) / 2).float()
    cam = torch.tensor([1.0, 0.0, 0.0, 0.0, *centre.tolist()], device=dev, requires_grad=True)
    opt = torch.optim.Adam([cam], lr=1e-3)
    bound = sc.bound.to(dev)
    E, H, W = args.edge, sc.H, sc.W

    def iteration():
        c2w = camera_from_tensor(cam)
        ro, rd, gd, gc, inside = sample_frames(E, H - E, E, W - E, args.pixels, sc.fx, sc.fy, sc.cx, sc.cy,
                                               c2w.unsqueeze(0), depth_d, color_d, bound=bound, device=dev)
        ro, rd, gd, gc = bbox_filter(ro, rd, gd, gc, inside)
        d, u, c, loss = r.render_batch_loss(grids, model, rd.float(), ro.float(), dev, "color", gd, gc,
                                            loss="tracker", color_term=True, w_color_loss=0.5,
                                            handle_dynamic=True)
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)
        return loss.item(), (ro.detach(), rd.detach(), gd, gc)

    for _ in range(args.warmup):
        iteration()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(args.iters):
        lv, rays = iteration()
    torch.cuda.synchronize()
    it_ms = (time.perf_counter() - t) / args.iters * 1e3
    # the render + loss + backward alone on the last iteration's rays (rays as leaves)
    ro, rd, gd, gc = rays
    ro, rd = ro.float().requires_grad_(True), rd.float().requires_grad_(True)

    def render_only():
        d, u, c, loss = r.render_batch_loss(grids, model, rd, ro, dev, "color", gd, gc, loss="tracker",
                                            color_term=True, w_color_loss=0.5, handle_dynamic=True)
        loss.backward()
        ro.grad = rd.grad = None
        return loss
    for _ in range(args.warmup):
        render_only()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(args.iters):
        render_only()
    torch.cuda.synchronize()
    rb_ms = (time.perf_counter() - t) / args.iters * 1e3
    graph = {}
    if args.graph:
        try:
            graph = graph_variant(args, r, grids, model, cam, sc, depth_d, color_d, bound, dev)
        except Exception as e:  # reported; the eager line stands
            graph = {"graph_error": repr(e)[:300]}
    print(json.dumps({**graph, "workload": f"{args.scene} Tracker iteration, {args.pixels} pixels (edge {args.edge}), "
                                  f"stage color, handle_dynamic, colour term", "rays_kept": int(ro.shape[0]),
                      "ms_per_iteration": round(it_ms, 4), "render_loss_backward_ms": round(rb_ms, 4),
                      "iterations_per_s": round(1e3 / it_ms, 1), "last_loss": lv}))


if __name__ == "__main__":
    main()
