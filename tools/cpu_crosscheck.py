"""CPU-baseline cross-check: time the oracle (bench.py's cpu_baseline,
``kind: "port"``) against the reference's own ``Renderer.render_batch_ray`` imported
from /root/reference, on the same C2 inputs, at equal thread counts, and compare
their outputs.  Runs only in the build container (the reference never travels to the
GPU box).  Writes profiles/cpu_crosscheck.json.

Both legs: render_batch_ray (stage color, 1000 rays x 48 samples, Replica room0) +
the Mapper's L1 loss (oracle.mapper_loss applied to either renderer's outputs) +
backward into rays, grids and decoder parameters (BA mode).

Usage:  python tools/cpu_crosscheck.py [--threads 8] [--iters 5]
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time
import types

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "nice-slam-annotation_amd"), os.path.join(REPO, "tests", "golden")]

from nicecore import scene as S  # noqa: E402
from oracle import nice_oracle as O  # noqa: E402
import make_golden as MG  # noqa: E402  (reference import harness)


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=os.cpu_count())
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--rays", type=int, default=1000)
    args = ap.parse_args()
    torch.set_num_threads(args.threads)

    ref_config, RefRenderer, cfg = MG._import_reference()
    sc = S.make_scene("replica_room0")
    torch.manual_seed(0)
    model = ref_config.get_model(cfg, nice=True)
    bound = sc.bound
    model.bound = bound
    for n in ("middle", "fine", "color"):
        getattr(model, n + "_decoder").bound = bound
    model.coarse_decoder.bound = bound * cfg['model']['coarse_bound_enlarge']
    grids = S.init_grids(sc.shapes, generator=torch.Generator().manual_seed(0))
    slam = types.SimpleNamespace(nice=True, bound=bound, H=sc.H, W=sc.W, fx=sc.fx, fy=sc.fy,
                                 cx=sc.cx, cy=sc.cy)
    ref = RefRenderer(cfg, None, slam)
    ro, rd, dep, col = S.synth_rays(sc, args.rays, seed=1000)
    dec_b = S.decoder_bounds(bound)
    prm = {k: v.detach().clone().requires_grad_(True) for k, v in model.named_parameters()}
    g_o = {k: v.clone().requires_grad_(True) for k, v in grids.items()}
    g_r = {k: v.clone().requires_grad_(True) for k, v in grids.items()}

    def leg_ref():
        model.zero_grad(set_to_none=True)
        for t in g_r.values():
            t.grad = None
        ro_, rd_ = ro.clone().requires_grad_(True), rd.clone().requires_grad_(True)
        d, u, c = ref.render_batch_ray(g_r, model, rd_, ro_, 'cpu', 'color', dep)
        O.mapper_loss(d, c, dep, col, 0.2, True).backward()
        return d, u, c, ro_.grad

    def leg_oracle():
        for t in list(prm.values()) + list(g_o.values()):
            t.grad = None
        ro_, rd_ = ro.clone().requires_grad_(True), rd.clone().requires_grad_(True)
        d, u, c = O.render_batch_ray(g_o, prm, dec_b, bound, rd_, ro_, 'color', dep)
        O.mapper_loss(d, c, dep, col, 0.2, True).backward()
        return d, u, c, ro_.grad

    def timed(fn):
        out = fn()  # warm-up
        ts = []
        for _ in range(args.iters):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        ts.sort()
        return out, ts[len(ts) // 2]

    # interleave the legs' timing so both see the same machine state
    (dr, ur, cr, gr), t_ref = timed(leg_ref)
    (do, uo, co, go), t_orc = timed(leg_oracle)
    _, t_ref2 = timed(leg_ref)
    t_ref = min(t_ref, t_ref2)

    def rel(a, b):
        a, b = a.detach().double(), b.detach().double()
        return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))

    res = {
        "config": f"C2 replica_room0 {args.rays} rays x 48 samples, stage color, mapper BA grads "
                  "(rays + grids + decoders), L1 mapper loss",
        "threads": args.threads, "cpu_model": cpu_model(), "torch": torch.__version__,
        "reference_ms_per_iter": round(1e3 * t_ref, 2), "oracle_ms_per_iter": round(1e3 * t_orc, 2),
        "reference_rays_s": round(args.rays / t_ref, 1), "oracle_rays_s": round(args.rays / t_orc, 1),
        "oracle_over_reference": round(t_ref / t_orc, 3),
        "max_rel_err": {"depth": rel(do, dr), "var": rel(uo, ur), "color": rel(co, cr),
                        "grad/rays_o": rel(go, gr),
                        "grad/grid_fine": rel(g_o["grid_fine"].grad, g_r["grid_fine"].grad),
                        "grad/color_decoder.output_linear.weight":
                            rel(prm["color_decoder.output_linear.weight"].grad,
                                model.color_decoder.output_linear.weight.grad)},
        "timing": f"median of {args.iters} iterations after one warm-up (reference: best of two medians)",
    }
    print(json.dumps(res, indent=1))
    out = os.path.join(REPO, "profiles", "cpu_crosscheck.json")
    with open(out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
