"""Diagnostic (GPU): where the per-element gate's largest HIP-only errors come from.
For one golden case: the decoder bias gradients that are plain sums of d raw over the
points (output_linear.bias of the occupancy decoders) against the float64 truth, and
the HIP eval_points raw occupancy against the oracle's float32 / float64 values on the
case's own sample points.  Run once per library variant (NICECORE_LIB=...)."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "nice-slam-annotation_amd"), os.path.join(REPO, "tests")):
    sys.path.insert(0, p)
from conftest import load_case, load_scene  # noqa: E402
from parity_common import build_model, case_stage, make_renderer, oracle_render_grads, run_case, scene_of  # noqa: E402
from oracle import nice_oracle as O  # noqa: E402

case = sys.argv[1] if len(sys.argv) > 1 else "color_depth"
rec, got = run_case(case, channels_last=True)
bound, cbound, grids, params = load_scene(scene_of(case))
stage, wd = case_stage(case)
dec_b = {"coarse": cbound, "middle": bound, "fine": bound, "color": bound}
gt = rec["gt_depth"] if wd else None
args = (grids, params, dec_b, bound, rec["rays_o"], rec["rays_d"], stage, gt, (rec["g_depth"], rec["g_var"], rec["g_color"]))
t = oracle_render_grads(*args, f64=True, round_inputs=True)
lib = os.environ.get("NICECORE_LIB", "default")
keys = sorted(k for k in t if k.startswith("grad/param/") and k.endswith(".bias")) + ["depth", "var"]
for k in keys:
    if k in t and k in got:
        tt = t[k].double()
        m = max(float(tt.abs().max()), 1e-300)
        print(f"{os.path.basename(lib)} {case} {k:46s}: hip-t {float((got[k].double() - tt).abs().max()) / m:.3e}  "
              f"ref-t {float((rec[k].double() - tt).abs().max()) / m:.3e}  (of |t| {m:.3e})")
# raw on the case's points
if "pts" not in rec:
    sys.exit(0)
pts = rec["pts"].double()
with torch.no_grad():
    r32 = O.eval_points(pts.clone(), grids, params, bound, dec_b, stage)
    with O.float64_mode(True):
        g64 = {k: v.double() for k, v in grids.items()}
        p64 = {k: v.double() for k, v in params.items()}
        r64 = O.eval_points(pts.clone(), g64, p64, bound, dec_b, stage)
    model = build_model(params, bound, cbound, "cuda")
    g = {k: v.cuda() for k, v in grids.items()}
    rh = make_renderer(bound).eval_points(pts.cuda(), model, g, stage, "cuda").cpu().double()
m = r64[:, 3].abs() < 99
for name, r in (("hip", rh), ("oracle32", r32.double())):
    e = (r[m, 3] - r64[m, 3]).abs()
    print(f"{os.path.basename(lib)} raw occ {name}: max {e.max():.3e} mean {e.mean():.3e} rel-to-max {e.max() / r64[m, 3].abs().max():.3e}")
