"""A/B bit-identity of two render-core libraries on the bench workloads.

A change that must not move a single bit (a different route to the same bytes, e.g. the
split-f16 weight images built once in global memory instead of in every forward
workgroup) is checked by running the same seeded C2 steps with both libraries and
comparing every output and gradient bit for bit.

    python tools/ab_bitident.py dump OUT.npz        # with the library NICECORE_LIB names (or in-tree)
    python tools/ab_bitident.py compare A.npz B.npz

Workloads: stages coarse / middle / fine / color on both grid layouts (channels_last runs
the fused-gather forward, ncdhw k_grid_gather + k_mlp_fwd), render + Mapper loss
+ backward, plus Renderer.eval_points (the points path).  The grid gradients are summed by
float atomics (order not fixed run to run): they are reported with their max difference
instead of failing.
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "nice-slam-annotation_amd"))


def dump(out):
    import torch
    import bench
    res = {}
    dev = torch.device("cuda:0")
    for layout in ("channels_last", "ncdhw"):
        for stage in ("coarse", "middle", "fine", "color"):
            sys.argv = ["bench.py", "--stage", stage, "--layout", layout, "--eager"]
            args = bench.parse()
            w = bench.build_workload(args, 0, dev)
            grids, model, renderer = w["grids"], w["model"], w["renderer"]
            ro, rd, gt, gtc = w["ro"], w["rd"], w["gt"], w["gtc"]
            depth, unc, color, loss = renderer.render_batch_loss(
                grids, model, rd, ro, dev, stage, gt, gtc, **bench.LOSS_KW["ba"](stage))
            loss.backward()
            torch.cuda.synchronize()
            tag = f"{layout}/{stage}/"
            for n, t in (("depth", depth), ("unc", unc), ("color", color), ("loss", loss), ("g_rays_o", ro.grad),
                         ("g_rays_d", rd.grad)):
                res[tag + n] = t.detach().cpu().numpy()
            for n, p in model.named_parameters():
                if p.grad is not None:
                    res[tag + "param/" + n] = p.grad.cpu().numpy()
            for k, g in grids.items():
                if g.grad is not None:
                    res[tag + "atomic/grid/" + k] = g.grad.cpu().numpy()
            with torch.no_grad():  # the points path (k_points_prep builds the images)
                pts = ro.detach()[:256] + 0.5 * rd.detach()[:256]
                raw = renderer.eval_points(pts, model, grids, stage=stage, device=dev)
            res[tag + "eval_points"] = raw.cpu().numpy()
            del w, grids, model, renderer
    np.savez(out, **res)
    print("dumped", len(res), "tensors to", out, flush=True)


def compare(a, b):
    A, B = np.load(a), np.load(b)
    bad = 0
    assert sorted(A.files) == sorted(B.files), "different tensor sets"
    for k in sorted(A.files):
        x, y = A[k], B[k]
        same = x.shape == y.shape and x.tobytes() == y.tobytes()
        if same:
            continue
        d = float(np.max(np.abs(x.astype(np.float64) - y.astype(np.float64))))
        m = float(np.max(np.abs(x.astype(np.float64)))) or 1.0
        atomic = "/atomic/" in k
        print(f"{'ORDER' if atomic else 'DIFF '} {k}: max |a-b| {d:.3e} ({d / m:.3e} of max)", flush=True)
        if not atomic:
            bad += 1
    print(f"{len(A.files)} tensors, {bad} not bit-identical (atomic-order tensors excluded)", flush=True)
    return bad == 0


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        dump(sys.argv[2])
    else:
        sys.exit(0 if compare(sys.argv[2], sys.argv[3]) else 1)
