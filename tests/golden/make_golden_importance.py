"""Golden vectors for hierarchical sampling inside render_batch_ray (N_importance > 0,
src/utils/Renderer.py:239-259) FROM THE REFERENCE ITSELF.  Build container only.

Same tiny scene, model and grids as make_golden.py (its setup()); the reference's
Renderer is built with rendering.N_importance = 8 (perturb = 0, so sample_pdf is
deterministic) and renders seeded rays; random upstream gradients are
back-propagated.  Stored: rays, outputs, all gradients.  Only numbers are written.

Usage:  python tests/golden/make_golden_importance.py
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import make_golden as MG  # noqa: E402
from nicecore import scene as S  # noqa: E402

STAGES = ["coarse", "middle", "fine", "color"]
CASES = [
    # name, stage, n_rays, with_depth, zero_frac, outside_frac, seed, N_importance
    ("imp_color_depth", "color", 20, True, 0.1, 0.2, 31, 8),
    ("imp_middle_nodepth", "middle", 16, False, 0.0, 0.2, 32, 12),
]


def main():
    ref_config, RefRenderer, cfg, scene, model, grids_big, bound, slam = MG.setup()
    for name, stage, n, with_depth, zf, of, seed, nimp in CASES:
        cfg['rendering']['N_importance'] = nimp
        renderer = RefRenderer(cfg, None, slam)
        ro, rd, dep, col = S.synth_rays(scene, n, n_poses=6, seed=seed, zero_depth_frac=zf, outside_frac=of)
        ro = ro.clone().requires_grad_(True)
        rd = rd.clone().requires_grad_(True)
        g = {k: v.clone().requires_grad_(True) for k, v in grids_big.items()}
        for p in model.parameters():
            p.grad = None
        depth, var, color = renderer.render_batch_ray(g, model, rd, ro, 'cpu', stage, dep if with_depth else None)
        gen2 = torch.Generator().manual_seed(seed + 100)
        gd = torch.randn(depth.shape, generator=gen2, dtype=torch.float64)
        gv = torch.randn(var.shape, generator=gen2, dtype=torch.float64) * 0.5
        gc = torch.randn(color.shape, generator=gen2, dtype=torch.float32)
        torch.autograd.backward([depth, var, color], [gd, gv, gc])
        rec = {"rays_o": ro.detach().numpy(), "rays_d": rd.detach().numpy(), "gt_depth": dep.numpy(),
               "depth": depth.detach().numpy(), "var": var.detach().numpy(), "color": color.detach().numpy(),
               "g_depth": gd.numpy(), "g_var": gv.numpy(), "g_color": gc.numpy(),
               "grad/rays_o": ro.grad.numpy(), "grad/rays_d": rd.grad.numpy(),
               "stage": np.array(STAGES.index(stage)), "with_depth": np.array(with_depth),
               "n_importance": np.array(nimp)}
        for k, v in g.items():
            if v.grad is not None:
                rec["grad/" + k] = v.grad.numpy()
        for pn, p in model.named_parameters():
            if p.grad is not None:
                rec["grad/param/" + pn] = p.grad.numpy()
        np.savez_compressed(os.path.join(HERE, f"case_{name}.npz"), **rec)
        print(name, depth[:3].tolist())


if __name__ == "__main__":
    main()
