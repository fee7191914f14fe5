"""Diagnostic (GPU): where the HIP importance-sampling render (N_importance > 0) departs from
the reference's golden vectors (tests/test_importance.py), ray by ray.

For each golden importance case: per ray, |HIP - reference| of depth and var (in units of
each tensor's max-abs), the second-pass sample depths of HIP (z_out) against the oracle's
own first pass + sample_pdf on the reference's float32 program, and the same deviations for
unit-permuted float32 oracles (another float32 implementation of the decoders).

    python tools/diag_importance.py
"""
import os
import sys
import types

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "nice-slam-annotation_amd"), os.path.join(REPO, "tests")):
    sys.path.insert(0, p)
from conftest import load_case, load_meta, load_scene  # noqa: E402
from parity_common import build_model, permuted_problem  # noqa: E402
from oracle import nice_oracle as O  # noqa: E402

meta = load_meta()
for name in ("imp_color_depth", "imp_middle_nodepth"):
    rec = load_case(name)
    stage = ["coarse", "middle", "fine", "color"][int(rec["stage"])]
    wd, nimp = bool(rec["with_depth"]), int(rec["n_importance"])
    bound, cbound, grids, params = load_scene()
    dec_b = {"coarse": cbound, "middle": bound, "fine": bound, "color": bound}
    gt = rec["gt_depth"] if wd else None
    from nicecore import scene as S
    from nicecore.renderer import Renderer
    model = build_model(params, bound, cbound, "cuda")
    g = {k: v.cuda().contiguous(memory_format=torch.channels_last_3d) for k, v in grids.items()}
    cfg = {"rendering": dict(S.DEFAULT_RENDERING, N_importance=nimp), "scale": 1, "occupancy": True}
    slam = types.SimpleNamespace(nice=True, bound=bound, H=48, W=64, fx=40.0, fy=40.0, cx=31.5, cy=23.5)
    with torch.no_grad():
        d, v, c = Renderer(cfg, None, slam).render_batch_ray(g, model, rec["rays_d"].cuda(), rec["rays_o"].cuda(),
                                                             "cuda", stage, gt.cuda() if gt is not None else None)
    d, v = d.cpu(), v.cpu()
    sd, sv = float(rec["depth"].abs().max()), float(rec["var"].abs().max())
    ed = (d - rec["depth"]).abs() / sd
    ev = (v - rec["var"]).abs() / sv
    print(f"[{name}] stage {stage}, {rec['rays_o'].shape[0]} rays, N_importance {nimp}")
    print(f"  HIP vs reference: depth max {float(ed.max()):.2e} (ray {int(ed.argmax())}), "
          f"var max {float(ev.max()):.2e} (ray {int(ev.argmax())}); rays over 2e-5: "
          f"{int(((ed > 2e-5) | (ev > 2e-5)).sum())}")
    top = torch.argsort(torch.maximum(ed, ev), descending=True)[:5]
    print("  worst rays:", ", ".join(f"{int(i)}: d {float(ed[i]):.1e} v {float(ev[i]):.1e}" for i in top))
    for seed in (1, 2, 3):
        g2, p2, _ = permuted_problem(grids, params, seed)
        with torch.no_grad():
            d2, v2, _ = O.render_batch_ray(g2, p2, dec_b, bound, rec["rays_d"], rec["rays_o"], stage, gt,
                                           meta["n_samples"], meta["n_surface"], n_importance=nimp)
        e2d = (d2 - rec["depth"]).abs() / sd
        e2v = (v2 - rec["var"]).abs() / sv
        print(f"  permuted float32 oracle {seed}: depth max {float(e2d.max()):.2e} var max {float(e2v.max()):.2e}; "
              f"on HIP's worst rays: " + ", ".join(f"{float(e2d[i]):.1e}/{float(e2v[i]):.1e}" for i in top[:3]))
