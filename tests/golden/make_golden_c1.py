"""Golden vectors at BASELINE.json configs[0] (C1), FROM THE REFERENCE ITSELF.

C1: Replica room0 (bound snapped by load_bound, middle grid [21, 28, 37]), 200 rays,
stage ``middle``, no render depth (S = 32 stratified samples), gradients to the rays,
grid_middle and the middle decoder.  Same harness as make_golden.py:
the reference's own modules (src.config get_model under torch.manual_seed(0),
src.utils.Renderer.render_batch_ray on the CPU, the decoder.py:340 CPU patch), random
upstream gradients.

Two cases:
  c1_room0        grids as grid_init leaves them (N(0, 0.01), src/NICE_SLAM.py:289-319) and
                  the decoders' own initialisers -- exactly the benchmark's C1 data
                  (bench.build_workload: init_grids seed 0, rays synth_rays seed 1000);
  c1_room0_spread the middle grid x30 and the middle occupancy bias at -0.55 (as
                  make_golden.py), so the compositing weights spread over all 32 samples.

The grids and decoder parameters are NOT stored: they are regenerated bit-identically from
their seeds (nicecore.scene.init_grids, nicecore.decoder.build_default_nice -- asserted
equal to the reference model's here).  Stored: rays, outputs, upstream and input
gradients (the grid gradient compressed: it is zero off the touched voxels).

Usage:  python tests/golden/make_golden_c1.py
"""
from __future__ import annotations

import json
import os
import sys
import types

import numpy as np
import torch

from make_golden import HERE, REPO, S, _import_reference

sys.path.insert(0, os.path.join(REPO, "tests"))
from parity_common import C1_CASES as CASES, c1_inputs as scene_inputs  # noqa: E402

N_RAYS = 200


def main():
    ref_config, RefRenderer, cfg = _import_reference()
    sc = S.make_scene("replica_room0")
    cfg['mapping']['bound'] = S.PRESETS["replica_room0"]["bound"]
    bound = torch.from_numpy(np.array(cfg['mapping']['bound']) * cfg['scale'])
    bd = cfg['grid_len']['bound_divisible']
    bound[:, 1] = (((bound[:, 1] - bound[:, 0]) / bd).int() + 1) * bd + bound[:, 0]  # load_bound
    assert torch.equal(bound, sc.bound), (bound, sc.bound)
    meta = {"scene": "replica_room0", "n_rays": N_RAYS, "stage": "middle", "cases": [], "torch": torch.__version__,
            "n_samples": cfg['rendering']['N_samples']}
    ro, rd, _, _ = S.synth_rays(sc, N_RAYS, seed=1000)
    for name, scale, bias, useed in CASES:
        torch.manual_seed(0)
        model = ref_config.get_model(cfg, nice=True)
        _, grids, params, _ = scene_inputs(name)
        with torch.no_grad():
            if bias is not None:
                model.middle_decoder.output_linear.bias.fill_(bias)
        for n, p in model.named_parameters():  # the regenerated parameters are the reference's
            assert torch.equal(p.detach(), params[n]), n
        model.bound = bound
        for n in ("middle", "fine", "color"):
            getattr(model, n + "_decoder").bound = bound
        model.coarse_decoder.bound = bound * cfg['model']['coarse_bound_enlarge']
        slam = types.SimpleNamespace(nice=True, bound=bound, H=sc.H, W=sc.W, fx=sc.fx, fy=sc.fy, cx=sc.cx, cy=sc.cy)
        renderer = RefRenderer(cfg, None, slam)
        r_o = ro.clone().requires_grad_(True)
        r_d = rd.clone().requires_grad_(True)
        g = {k: v.clone().requires_grad_(True) for k, v in grids.items()}
        depth, var, color = renderer.render_batch_ray(g, model, r_d, r_o, 'cpu', 'middle', None)
        gen = torch.Generator().manual_seed(useed)
        gd = torch.randn(depth.shape, generator=gen, dtype=torch.float64)
        gv = torch.randn(var.shape, generator=gen, dtype=torch.float64) * 0.5
        gc = torch.randn(color.shape, generator=gen, dtype=torch.float32)
        torch.autograd.backward([depth, var, color], [gd, gv, gc])
        rec = {"rays_o": ro.numpy(), "rays_d": rd.numpy(),
               "depth": depth.detach().numpy(), "var": var.detach().numpy(), "color": color.detach().numpy(),
               "g_depth": gd.numpy(), "g_var": gv.numpy(), "g_color": gc.numpy(),
               "grad/rays_o": r_o.grad.numpy(), "grad/rays_d": r_d.grad.numpy()}
        for k, v in g.items():
            if v.grad is not None:
                rec["grad/" + k] = v.grad.numpy()
        for pn, p in model.named_parameters():
            if p.grad is not None:
                rec["grad/param/" + pn] = p.grad.numpy()
        np.savez_compressed(os.path.join(HERE, f"case_{name}.npz"), **rec)
        meta["cases"].append(dict(name=name, stage="middle", n_rays=N_RAYS, with_depth=False))
        touched = int((g["grid_middle"].grad.abs().amax(1) > 0).sum())
        print(f"{name}: depth[:3]={depth[:3].tolist()} touched middle voxels {touched} "
              f"grads {sorted(k for k in rec if k.startswith('grad/'))[:4]}...")
    with open(os.path.join(HERE, "c1_meta.json"), "w") as f:
        json.dump(meta, f, indent=1)


if __name__ == "__main__":
    main()
