"""A whole Tracker iteration on the drop-ins (SURVEY.md §8f rank 2 with the render path):
Tracker.optimize_cam_in_batch (src/Tracker.py:78-135) for Replica room0 — camera tensor
(quaternion + translation, common.py:163-176) -> c2w, 200 pixels sampled on the device
from a resident depth / colour frame (nicecore.sampling.sample_frames: rays, gt and the
bbox pre-filter mask in one launch, Tracker.py:98-111), the boolean compaction of the
reference (one host sync for the count) -- or, in the graph variant, the same filter as the
core's per-ray mask (ray_mask, ABI v10: no compaction, no sync) --, render_batch_ray + the tracker loss
(handle_dynamic, colour term, w_color_loss 0.5; Tracker.py:113-130) fused in the core,
backward to the camera tensor (the pose-gradient launch), Adam step, loss.item().

The resident frame's depth reaches past the bound on part of the image (--far), so a
share of the rays fails the pre-filter every iteration (reported as rays_kept).

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


def quad2rotation(q):
    """common.py:137-160 for one quaternion [qr, qi, qj, qk]: R with two_s = 2 / |q|^2,
    so a quaternion Adam has moved off unit norm maps to the reference's rotation."""
    qr, qi, qj, qk = q[0], q[1], q[2], q[3]
    two_s = 2.0 / (q * q).sum(-1)
    return torch.stack([
        torch.stack([1 - two_s * (qj ** 2 + qk ** 2), two_s * (qi * qj - qk * qr), two_s * (qi * qk + qj * qr)]),
        torch.stack([two_s * (qi * qj + qk * qr), 1 - two_s * (qi ** 2 + qk ** 2), two_s * (qj * qk - qi * qr)]),
        torch.stack([two_s * (qi * qk - qj * qr), two_s * (qj * qk + qi * qr), 1 - two_s * (qi ** 2 + qj ** 2)]),
    ])


def camera_from_tensor(q):
    """get_camera_from_tensor (common.py:163-176): [qr, qi, qj, qk, tx, ty, tz] -> [3, 4]
    c2w = [quad2rotation(quad) | T]."""
    return torch.cat([quad2rotation(q[:4]), q[4:7].reshape(3, 1)], dim=1)


def graph_variant(args, r, grids, model, cam, sc, depth_d, color_d, bound, dev):
    """The same iteration replayed as one hipGraph (nicecore.graph.GraphedStep, Adam
    capturable) with the loss read back once per iteration.  The pre-filter is the core's
    per-ray mask (render_batch_loss(ray_mask=inside)), so any frame replays without a
    compaction.  Checked first, eagerly at the start camera: the masked loss and camera
    gradient against the reference's compacted batch (rays[inside])."""
    from nicecore.graph import GraphedStep
    from nicecore.sampling import bbox_filter, sample_frames
    E, H, W = args.edge, sc.H, sc.W
    kw = dict(loss="tracker", color_term=True, w_color_loss=0.5, handle_dynamic=True)

    def rays_at(cm):
        c2w = camera_from_tensor(cm)
        torch.manual_seed(1234)  # the same pixels for both forms of the check
        return sample_frames(E, H - E, E, W - E, args.pixels, sc.fx, sc.fy, sc.cx, sc.cy,
                             c2w.unsqueeze(0), depth_d, color_d, bound=bound, device=dev)
    check = {}
    for form in ("masked", "compacted"):
        cm = cam.detach().clone().requires_grad_(True)
        ro, rd, gd, gc, inside = rays_at(cm)
        if form == "masked":
            loss = r.render_batch_loss(grids, model, rd, ro, dev, "color", gd, gc, **kw, ray_mask=inside)[3]
        else:
            ro, rd, gd, gc = bbox_filter(ro, rd, gd, gc, inside)
            loss = r.render_batch_loss(grids, model, rd, ro, dev, "color", gd, gc, **kw)[3]
        loss.backward()
        check[form] = (float(loss), cm.grad.detach().clone(), float(inside.float().mean()))
    (lm, gm, kept), (lc, gcam, _) = check["masked"], check["compacted"]
    gerr = float((gm - gcam).abs().max() / gcam.abs().max().clamp_min(1e-30))
    if not (abs(lm - lc) <= 1e-9 * max(abs(lc), 1.0) and gerr <= 1e-6):
        return {"graph_error": f"masked != compacted: loss {lm} vs {lc}, camera grad rel err {gerr}"}

    cam_g = cam.detach().clone().requires_grad_(True)
    opt_g = torch.optim.Adam([cam_g], lr=1e-3, capturable=True)

    def body():
        cam_g.grad = None
        c2w = camera_from_tensor(cam_g)
        ro, rd, gd, gc, inside = sample_frames(E, H - E, E, W - E, args.pixels, sc.fx, sc.fy, sc.cx, sc.cy,
                                               c2w.unsqueeze(0), depth_d, color_d, bound=bound, device=dev)
        d, u, c, loss = r.render_batch_loss(grids, model, rd, ro, dev, "color", gd, gc, **kw, ray_mask=inside)
        loss.backward()
        opt_g.step()
        return loss, inside.sum()
    def run(step):
        for _ in range(args.warmup):
            step()[0].item()
        torch.cuda.synchronize()
        kept_total = torch.zeros((), device=dev, dtype=torch.int64)
        t = time.perf_counter()
        for _ in range(args.iters):
            loss, nk = step()
            lg = loss.item()  # the Tracker's loss.item() sync, once per iteration
            kept_total += nk
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / args.iters * 1e3, lg, float(kept_total) / (args.iters * args.pixels)

    g_ms, lg, kf = run(GraphedStep(body))
    out = {"graph_ms_per_iteration": round(g_ms, 4), "graph_last_loss": lg, "graph_rays_kept_frac": round(kf, 4),
           "mask_check": {"loss_masked": lm, "loss_compacted": lc, "camera_grad_rel_err": gerr,
                          "rays_kept_frac": round(kept, 4)}}
    # the fused form: camera tensor -> rays inside the sampling kernel and d camera inside the
    # pose-gradient kernel (sample_frames_from_tensor, ABI v11), the 7-float Adam as one
    # k_adam_multi launch (nicecore.optim.Adam, capturable) -- checked first against the
    # torch-ops form on one eager iteration from the same camera
    from nicecore.optim import Adam as NcAdam
    from nicecore.sampling import sample_frames_from_tensor
    ref_cam = cam.detach().clone().requires_grad_(True)
    fus_cam = cam.detach().clone().requires_grad_(True)
    for cm, fused in ((ref_cam, False), (fus_cam, True)):
        torch.manual_seed(4321)
        if fused:
            ro, rd, gd, gc, inside = sample_frames_from_tensor(E, H - E, E, W - E, args.pixels, sc.fx, sc.fy, sc.cx,
                                                               sc.cy, cm, depth_d, color_d, bound=bound, device=dev)
        else:
            ro, rd, gd, gc, inside = sample_frames(
                E, H - E, E, W - E, args.pixels, sc.fx, sc.fy, sc.cx, sc.cy, camera_from_tensor(cm).unsqueeze(0),
                depth_d, color_d, bound=bound, device=dev)
        r.render_batch_loss(grids, model, rd, ro, dev, "color", gd, gc, **kw, ray_mask=inside)[3].backward()
    ferr = float((fus_cam.grad - ref_cam.grad).abs().max() / ref_cam.grad.abs().max().clamp_min(1e-30))
    cam_f = cam.detach().clone().requires_grad_(True)
    opt_f = NcAdam([cam_f], lr=1e-3, capturable=True)

    def body_fused():
        cam_f.grad = None
        ro, rd, gd, gc, inside = sample_frames_from_tensor(E, H - E, E, W - E, args.pixels, sc.fx, sc.fy, sc.cx,
                                                           sc.cy, cam_f, depth_d, color_d, bound=bound, device=dev)
        d, u, c, loss = r.render_batch_loss(grids, model, rd, ro, dev, "color", gd, gc, **kw, ray_mask=inside)
        loss.backward()
        opt_f.step()
        return loss, inside.sum()
    f_ms, lf, kff = run(GraphedStep(body_fused))
    out.update({"graph_fused_ms_per_iteration": round(f_ms, 4), "graph_fused_last_loss": lf,
                "graph_fused_rays_kept_frac": round(kff, 4), "fused_camera_grad_rel_err_vs_torch_ops": ferr})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--pixels", type=int, default=200)
    ap.add_argument("--edge", type=int, default=100)
    ap.add_argument("--scene", default="replica_room0")
    ap.add_argument("--graph", action="store_true",
                    help="also replay the iteration as one hipGraph (the pre-filter as the core's per-ray "
                         "mask, checked against the compacted batch)")
    ap.add_argument("--far", type=float, default=5.5,
                    help="frame depth ~ U(0.5, far) m: past the bound's exit on part of the image, so part "
                         "of the rays fail the pre-filter (2.5 or less keeps every ray from the room centre)")
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
    depth = torch.rand(sc.H, sc.W, generator=gen) * (args.far - 0.5) + 0.5
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
    kept = 0
    for _ in range(args.iters):
        lv, rays = iteration()
        kept += rays[0].shape[0]
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
                      "rays_kept_frac": round(kept / (args.iters * args.pixels), 4),
                      "ms_per_iteration": round(it_ms, 4), "render_loss_backward_ms": round(rb_ms, 4),
                      "iterations_per_s": round(1e3 / it_ms, 1), "last_loss": lv}))


if __name__ == "__main__":
    main()
