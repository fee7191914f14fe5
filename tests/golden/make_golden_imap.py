"""Golden vectors for the iMAP* render path FROM THE REFERENCE ITSELF (build container only).

Imports the reference's own modules (src.config.load_config / get_model(nice=False),
src.utils.Renderer with ``slam.nice = False``), loads configs/Replica/room0_imap.yaml
(occupancy: False, N_samples 32, N_surface 0, N_importance 12), renders seeded
synthetic rays of the tiny scene through ``Renderer.render_batch_ray`` on the CPU,
back-propagates random upstream gradients and stores inputs / outputs / gradients as
.npz fixtures (imap_*.npz) next to this script.  Only numeric vectors are written.
No harness patch is needed: the iMAP* path never builds a 'cuda:' device string.

Usage:  python tests/golden/make_golden_imap.py
"""
from __future__ import annotations

import json
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("NICE_REF", "/root/reference")
sys.path.insert(0, os.path.join(REPO, "nice-slam-annotation_amd"))

from nicecore import scene as S  # noqa: E402

CASES = [
    # name, n_rays, with_depth, N_importance, zero_frac, outside_frac, seed
    ("depth_imp", 24, True, 12, 0.15, 0.25, 31),
    ("depth_noimp", 20, True, 0, 0.1, 0.2, 32),
    ("nodepth_imp", 16, False, 12, 0.0, 0.25, 33),
]


def main():
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    cwd = os.getcwd()
    os.chdir(REF)
    from src import config as ref_config
    from src.utils.Renderer import Renderer as RefRenderer
    cfg = ref_config.load_config('configs/Replica/room0_imap.yaml', 'configs/imap.yaml')
    os.chdir(cwd)
    assert cfg['occupancy'] is False and cfg['rendering']['N_surface'] == 0

    scene = S.make_scene("tiny")
    torch.manual_seed(0)
    model = ref_config.get_model(cfg, nice=False)
    # random init gives sigma ~ 0: bias the density head so weights spread along the rays
    with torch.no_grad():
        model.output_linear.bias[3] = 3.0
    bound = scene.bound
    slam = types.SimpleNamespace(nice=False, bound=bound, H=scene.H, W=scene.W, fx=scene.fx,
                                 fy=scene.fy, cx=scene.cx, cy=scene.cy)
    renderer = RefRenderer(cfg, None, slam)
    sc = {"bound": bound.numpy(), **{"param/" + n: p.detach().numpy() for n, p in model.named_parameters()}}
    np.savez_compressed(os.path.join(HERE, "imap_scene.npz"), **sc)
    meta = {"scene": "tiny", "cases": [], "torch": torch.__version__,
            "config": "configs/Replica/room0_imap.yaml", "n_samples": cfg['rendering']['N_samples']}
    for name, n, with_depth, n_imp, zf, of, seed in CASES:
        renderer.N_importance = n_imp
        ro, rd, dep, _ = S.synth_rays(scene, n, n_poses=6, seed=seed, zero_depth_frac=zf, outside_frac=of)
        ro = ro.clone().requires_grad_(True)
        rd = rd.clone().requires_grad_(True)
        for p in model.parameters():
            p.grad = None
        seen = []
        orig_eval = renderer.eval_points

        def recording_eval(p, decoders, c=None, stage='color', device='cuda:0'):
            seen.append(p.detach().clone())
            return orig_eval(p, decoders, c, stage, device)

        renderer.eval_points = recording_eval
        gt = dep if with_depth else None
        depth, var, color = renderer.render_batch_ray(None, model, rd, ro, 'cpu', 'color', gt)
        renderer.eval_points = orig_eval
        gen2 = torch.Generator().manual_seed(seed + 100)
        gd = torch.randn(depth.shape, generator=gen2, dtype=torch.float64)
        gv = torch.randn(var.shape, generator=gen2, dtype=torch.float64) * 0.5
        gc = torch.randn(color.shape, generator=gen2, dtype=torch.float32)
        torch.autograd.backward([depth, var, color], [gd, gv, gc])
        rec = {"rays_o": ro.detach().numpy(), "rays_d": rd.detach().numpy(), "gt_depth": dep.numpy(),
               "depth": depth.detach().numpy(), "var": var.detach().numpy(), "color": color.detach().numpy(),
               "g_depth": gd.numpy(), "g_var": gv.numpy(), "g_color": gc.numpy(),
               "grad/rays_o": ro.grad.numpy(), "grad/rays_d": rd.grad.numpy()}
        for pn, p in model.named_parameters():
            rec["grad/param/" + pn] = p.grad.numpy()
        pts = seen[-1]
        with torch.no_grad():
            raw = renderer.eval_points(pts, model, None, 'color', 'cpu')
        rec["pts"], rec["raw"] = pts.numpy(), raw.numpy()
        np.savez_compressed(os.path.join(HERE, f"imap_{name}.npz"), **rec)
        meta["cases"].append(dict(name=name, n_rays=n, with_depth=with_depth, n_importance=n_imp))
        print(f"{name}: depth[:3]={depth[:3].tolist()} raw3 mean {raw[:, 3].mean():.3f}")
    with open(os.path.join(HERE, "imap_meta.json"), "w") as f:
        json.dump(meta, f, indent=1)


if __name__ == "__main__":
    main()
