"""Golden vectors for the stratified-sampling options of render_batch_ray FROM THE
REFERENCE ITSELF: ``lindisp`` (src/utils/Renderer.py:208-209) and ``perturb > 0``
(:211-219), which every shipped config leaves off but the Renderer supports.

Same harness as make_golden.py (the reference's Renderer and get_model on the tiny scene,
NICE.forward re-bound to allocate on p.device).  The reference draws the perturbation
with ``torch.rand(z_vals.shape)`` inside render_batch_ray -- the only draw of the global
generator in that call -- so the generator is seeded right before the call and the same
draws are recomputed afterwards from that seed and stored as ``t_rand``.
Zero-depth rays are left out of the lindisp cases: their near plane is 0, 1./near is
inf and the reference's depths become NaN there.

Usage:  python tests/golden/make_golden_strat.py
"""
from __future__ import annotations

import json
import os

import numpy as np
import torch

from make_golden import HERE, S, setup

CASES = [
    # name, stage, n_rays, with_depth, zero_frac, outside_frac, seed, lindisp, perturb
    ("strat_lindisp_color_depth", "color", 20, True, 0.0, 0.2, 41, True, 0.0),
    ("strat_perturb_color_depth", "color", 20, True, 0.15, 0.2, 42, False, 1.0),
    ("strat_lindisp_perturb_middle_nodepth", "middle", 16, False, 0.0, 0.25, 43, True, 1.0),
    ("strat_lindisp_perturb_fine_depth", "fine", 16, True, 0.0, 0.0, 44, True, 1.0),
]


def main():
    ref_config, RefRenderer, cfg, scene, model, grids_big, bound, slam = setup()
    renderer = RefRenderer(cfg, None, slam)
    meta = {"scene": "tiny", "cases": [], "torch": torch.__version__,
            "n_samples": cfg['rendering']['N_samples'], "n_surface": cfg['rendering']['N_surface']}
    for name, stage, n, with_depth, zf, of, seed, lindisp, perturb in CASES:
        renderer.lindisp, renderer.perturb = lindisp, perturb
        ro, rd, dep, col = S.synth_rays(scene, n, n_poses=6, seed=seed, zero_depth_frac=zf, outside_frac=of)
        ro = ro.clone().requires_grad_(True)
        rd = rd.clone().requires_grad_(True)
        g = {k: v.clone().requires_grad_(True) for k, v in grids_big.items()}
        for p in model.parameters():
            p.grad = None
        gt = dep if with_depth else None
        torch.manual_seed(1000 + seed)
        depth, var, color = renderer.render_batch_ray(g, model, rd, ro, 'cpu', stage, gt)
        torch.manual_seed(1000 + seed)
        t_rand = torch.rand(n, cfg['rendering']['N_samples']) if perturb > 0 else None
        gen2 = torch.Generator().manual_seed(seed + 100)
        gd = torch.randn(depth.shape, generator=gen2, dtype=torch.float64)
        gv = torch.randn(var.shape, generator=gen2, dtype=torch.float64) * 0.5
        gc = torch.randn(color.shape, generator=gen2, dtype=torch.float32)
        torch.autograd.backward([depth, var, color], [gd, gv, gc])
        assert torch.isfinite(depth).all() and torch.isfinite(var).all()
        rec = {
            "rays_o": ro.detach().numpy(), "rays_d": rd.detach().numpy(),
            "gt_depth": dep.numpy(), "gt_color": col.numpy(),
            "depth": depth.detach().numpy(), "var": var.detach().numpy(),
            "color": color.detach().numpy(),
            "g_depth": gd.numpy(), "g_var": gv.numpy(), "g_color": gc.numpy(),
            "grad/rays_o": ro.grad.numpy(), "grad/rays_d": rd.grad.numpy(),
        }
        if t_rand is not None:
            rec["t_rand"] = t_rand.numpy()
        for k, v in g.items():
            if v.grad is not None:
                rec["grad/" + k] = v.grad.numpy()
        for pn, p in model.named_parameters():
            if p.grad is not None:
                rec["grad/param/" + pn] = p.grad.numpy()
        np.savez_compressed(os.path.join(HERE, f"case_{name}.npz"), **rec)
        meta["cases"].append(dict(name=name, stage=stage, n_rays=n, with_depth=with_depth, lindisp=lindisp,
                                  perturb=perturb))
        print(f"{name}: depth[:3]={depth[:3].tolist()}")
    with open(os.path.join(HERE, "strat_meta.json"), "w") as f:
        json.dump(meta, f, indent=1)


if __name__ == "__main__":
    main()
