"""Forward-only point queries at Mesher scale: Mesher.eval_points
(Mesher.py:367-429) over the resolution^3 lattice of Mesher.get_grid_uniform
(Mesher.py:443-472: marching_cubes_bound widened by 0.05 on every side, so the points
past the renderer bound take the masked path too), split into
points_batch_size chunks, first at stage 'fine' (occupancy for marching cubes,
Mesher.py:569-575) and then at stage 'color' (vertex colours, Mesher.py:655-666).
Runs through nicecore's Renderer.eval_points (same mask rule: out-of-bound occupancy
100).  Prints points/s per stage; with --cpu-points N also times the CPU oracle's
eval_points (torch, all host threads) on the first N points.

    python tools/bench_mesher_query.py [--res 256] [--reps 3] [--cpu-points 200000]
"""
import argparse
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "nice-slam-annotation_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--res", type=int, default=256)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--batch", type=int, default=500000, help="Mesher points_batch_size")
    ap.add_argument("--scene", default="replica_room0")
    ap.add_argument("--cpu-points", type=int, default=0)
    args = ap.parse_args()
    import bench
    ns = argparse.Namespace(scene=args.scene, layout="channels_last", rays=16, mode="tracker",
                            sparse_grads="off", fix_fine=False, frustum="off")
    w = bench.build_workload(ns, 0, "cuda")
    sc, r, model = w["sc"], w["renderer"], w["model"]
    grids = {k: v.detach() for k, v in w["grids"].items()}
    r.points_batch_size = args.batch
    from nicecore.scene import mesher_lattice
    pts = mesher_lattice(sc.marching_cubes_bound, args.res)
    pts_d = pts.cuda()
    b = sc.bound
    inside = ((pts[:, 0] > b[0, 0]) & (pts[:, 0] < b[0, 1]) & (pts[:, 1] > b[1, 0]) & (pts[:, 1] < b[1, 1]) &
              (pts[:, 2] > b[2, 0]) & (pts[:, 2] < b[2, 1]))
    out = {"workload": f"{args.scene} Mesher.get_grid_uniform lattice {args.res}^3 = {pts.shape[0]} points "
                       f"(marching_cubes_bound +- 0.05, {100 * (1 - float(inside.double().mean())):.1f}% outside "
                       f"the renderer bound), points_batch_size {args.batch}, forward only"}
    with torch.no_grad():
        for stage in ("fine", "color"):
            r.eval_points(pts_d, model, grids, stage, "cuda")
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(args.reps):
                raw = r.eval_points(pts_d, model, grids, stage, "cuda")
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t) / args.reps
            assert raw.shape == (pts.shape[0], 4) and bool(torch.isfinite(raw).all())
            out[stage] = {"ms_per_lattice": round(dt * 1e3, 2),
                          "points_per_s": round(pts.shape[0] / dt, 1)}
        if args.cpu_points:
            from oracle import nice_oracle as O
            torch.set_num_threads(min(os.cpu_count() or 1, 16))
            params = O.params_from_module(model.cpu())
            gc = {k: v.cpu().contiguous() for k, v in grids.items()}
            dec_bounds = {"coarse": sc.bound * 2, "middle": sc.bound, "fine": sc.bound,
                          "color": sc.bound}
            p = pts[:args.cpu_points]
            t = time.perf_counter()
            O.eval_points(p, gc, params, sc.bound, dec_bounds, "color")
            cdt = time.perf_counter() - t
            out["cpu_oracle_color_points_per_s"] = round(p.shape[0] / cdt, 1)
            out["cpu_threads"] = torch.get_num_threads()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
