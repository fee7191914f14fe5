"""Diagnostic (CPU): does the split-f16 forward's activation representation explain the
per-element gate's remaining excess on a golden case?

k_mlp_fwd feeds every hidden layer its input as x = hi + 2^-11 lo, two round-to-nearest
f16 planes (nc_device.h split8): 23 significant bits where float32 keeps 24, so each
layer input carries up to one float32 ulp of extra rounding.  The weights are exact
(three planes) and every sum is float32.  This tool runs the float32 oracle with the
same rounding applied to every layer input (straight-through: the backward is the plain
float32 one) and scores it, the plain float32 oracle, and nothing else, against the
float64 truth with the gate of tests/test_gpu_elementwise.py.  If the emulation fails the
gate where the HIP path does, the excess is the representation, not an indexing or
ordering defect.

    python tools/diag_split_emulation.py fine_depth
"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "nice-slam-annotation_amd"), os.path.join(REPO, "tests")):
    sys.path.insert(0, p)
from conftest import load_case, load_scene  # noqa: E402
from parity_common import (case_stage, elementwise_vs_truth, oracle_render_grads,  # noqa: E402
                           oracle_render_grads_permuted, scene_of)
from oracle import nice_oracle as O  # noqa: E402

case = sys.argv[1] if len(sys.argv) > 1 else "fine_depth"
rec = load_case(case)
bound, cbound, grids, params = load_scene(scene_of(case))
stage, wd = case_stage(case)
dec_b = {"coarse": cbound, "middle": bound, "fine": bound, "color": bound}
gt = rec["gt_depth"] if wd else None
args = (grids, params, dec_b, bound, rec["rays_o"], rec["rays_d"], stage, gt,
        (rec["g_depth"], rec["g_var"], rec["g_color"]))
truth = oracle_render_grads(*args, f64=True, round_inputs=True)
truth = {k: v for k, v in truth.items() if k in rec}
p1 = oracle_render_grads_permuted(*args, seed=1)
p2 = oracle_render_grads_permuted(*args, seed=2)
plain = oracle_render_grads(*args)

_lin0 = O._lin


def _split23(x):
    if x.dtype != torch.float32:
        return x
    h = x.half().float()
    r = h + ((x - h) * 2048.0).half().float() / 2048.0
    return x + (r - x).detach()


def _lin_split(x, prm, name):
    return _lin0(x if name.endswith("output_linear") else _split23(x), prm, name)


O._lin = _lin_split
try:
    emu = oracle_render_grads(*args)
finally:
    O._lin = _lin0

refs = [rec, p1, p2]
for label, got in (("float32 oracle", plain), ("float32 oracle, split-f16 layer inputs", emu)):
    res = elementwise_vs_truth(got, refs, truth)
    bad = {k: v for k, v in res.items() if v["worst"] > 1}
    worst = max(v["worst"] for v in res.values())
    print(f"[{case}] {label}: worst ratio {worst:.3g}, tensors over the gate {len(bad)}")
    for k, v in sorted(res.items(), key=lambda kv: -kv[1]["worst"])[:6]:
        print(f"   {k:46s} worst {v['worst']:.3g} n_bad {v['n_bad']}/{v['n']}  l2 {v['l2_hip']:.2e} / {v['l2_ref']:.2e}")
