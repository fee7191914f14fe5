"""iMAP* (SURVEY.md §8f rank 4): one Mapper iteration of configs/imap.yaml on the HIP core.

Mapper.optimize_map with nice=False (Mapper.py:598-625): render_batch_ray over
``pixels = 5000`` rays (N_samples 32 + N_importance 12, N_surface 0, volume density),
L1 depth loss + w_color_loss * L1 colour loss, backward into all 222,747 MLP
parameters.  Synthetic rays on the Replica room0 bound, random-init MLP.  Prints one
JSON line: ms/iteration, rays/s, per-kernel HIP-event times, MFMA roofline of the
layer GEMMs; with --cpu-rays N also the CPU oracle (all host threads) on N rays.

    python tools/bench_imap.py [--rays 5000] [--steps 20] [--mode mapper|tracker] [--cpu-rays 200]
"""
import argparse
import json
import os
import sys
import time
import types

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "nice-slam-annotation_amd")]

F32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md, dense f32 MFMA
SPLIT16_PEAK_TFLOPS = 2500.0 / 3  # dense f16 MFMA / 3 products per split-f16 product (k_imap_gemm_h)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rays", type=int, default=5000)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--mode", default="mapper", choices=["mapper", "tracker"])
    ap.add_argument("--cpu-rays", type=int, default=0)
    args = ap.parse_args()
    from nicecore import _lib as L
    from nicecore import decoder as D
    from nicecore import scene as S
    from nicecore.renderer import Renderer
    sc = S.make_scene("replica_room0")
    m = D.build_imap(seed=0).cuda()
    with torch.no_grad():
        m.output_linear.bias[3] = 3.0
    cfg = {"rendering": {"lindisp": False, "perturb": 0.0, "N_samples": 32, "N_surface": 0, "N_importance": 12},
           "scale": 1, "occupancy": False}
    slam = types.SimpleNamespace(nice=False, bound=sc.bound, H=sc.H, W=sc.W, fx=sc.fx, fy=sc.fy, cx=sc.cx, cy=sc.cy)
    r = Renderer(cfg, None, slam)
    ro, rd, dep, col = S.synth_rays(sc, args.rays, seed=1)
    ro, rd, dep, col = ro.cuda(), rd.cuda(), dep.cuda(), col.cuda()
    tracker = args.mode == "tracker"
    for p in m.parameters():
        p.requires_grad_(not tracker)
    w_col = 0.5 if tracker else 0.05  # configs/imap.yaml:35, :62

    def step():
        rog = ro.requires_grad_(tracker)
        rdg = rd.requires_grad_(tracker)
        d, v, c = r.render_batch_ray(None, m, rdg, rog, "cuda", "color", dep)
        # Mapper.py:603-612 / Tracker.py:117-131 L1 terms; the depth mask as a where (no
        # boolean-index host sync inside the timed step)
        loss = torch.where(dep > 0, (dep - d).abs(), 0.).sum() + w_col * (col - c).abs().sum()
        loss.backward()
        for p in m.parameters():
            p.grad = None

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    with L.KernelTimer(["k_imap_gemm", "k_imap_fourier", "k_ray_setup", "k_composite_fwd",
                        "k_composite_bwd", "k_ray_grads", "k_sample_pdf"]) as kt:
        step()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / args.steps
    P = args.rays * 44
    P1 = args.rays * 32
    macs = 93 * 256 + 3 * 256 * 256 + 256 * 4
    gemm_ms = kt.result.get("k_imap_gemm", (0.0, 0))[0]
    # forward over both passes; backward dX (+ dW in mapper mode) over the second pass
    flops = 2 * macs * (P1 + P) + 2 * macs * P * (1 if tracker else 2)
    out = {"workload": f"iMAP* {args.mode} iteration, room0 bound, {args.rays} rays x (32 + 12 importance), "
                       f"MLP 93-256x4-4 f32", "ms_per_step": round(dt * 1e3, 4),
           "rays_per_s": round(args.rays / dt, 1),
           "kernels_ms": {k: round(v[0], 4) for k, v in kt.result.items()},
           "gemm_launches": kt.result.get("k_imap_gemm", (0, 0))[1],
           "gemm_tflops": round(flops / (gemm_ms * 1e-3) / 1e12, 2) if gemm_ms else None,
           "mfma_peak_tflops": F32_MFMA_PEAK_TFLOPS}
    if out["gemm_tflops"]:
        out["gemm_frac"] = round(out["gemm_tflops"] / F32_MFMA_PEAK_TFLOPS, 3)
        out["gemm_kernel"] = "k_imap_gemm (f32 MFMA)" if os.environ.get("NC_IMAP_F32") == "1" else \
            "k_imap_gemm_h (split-f16 MFMA; N < 64 layers on k_imap_gemm)"
        out["gemm_frac_split16_peak"] = round(out["gemm_tflops"] / SPLIT16_PEAK_TFLOPS, 3)
    if args.cpu_rays:
        from oracle import imap_oracle as IO
        torch.set_num_threads(min(os.cpu_count() or 1, 16))
        prm = {k: v.detach().cpu().clone().requires_grad_(not tracker) for k, v in m.named_parameters()}
        n = args.cpu_rays
        roc, rdc, dc = ro[:n].cpu(), rd[:n].cpu(), dep[:n].cpu()
        t = time.perf_counter()
        d, v, c = IO.render_batch_ray(prm, sc.bound, rdc.requires_grad_(tracker), roc.requires_grad_(tracker), dc,
                                      32, 12)
        (d.sum() + c.sum()).backward()
        cdt = time.perf_counter() - t
        out["cpu_baseline"] = {"rays_per_s": round(n / cdt, 1), "rays": n, "threads": torch.get_num_threads(),
                               "kind": "port"}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
