"""Diagnostic (CPU): how far legitimate float32 implementations reach into the per-element
gate of tests/test_gpu_elementwise.py on one golden case.  Each extra implementation is the
float32 oracle on the network with hidden units, Fourier features and grid channels
permuted (parity_common.permuted_problem, seeds 3..), scored exactly as the HIP path is:
against the float64 truth with references [reference vectors, permutation 1, permutation 2].

    python tools/gate_spread.py fine_depth [n_seeds]
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "nice-slam-annotation_amd"), os.path.join(REPO, "tests")):
    sys.path.insert(0, p)
from conftest import load_case, load_scene  # noqa: E402
from parity_common import (case_stage, elementwise_vs_truth, oracle_render_grads,  # noqa: E402
                           oracle_render_grads_permuted, scene_of)

case = sys.argv[1] if len(sys.argv) > 1 else "fine_depth"
n_seeds = int(sys.argv[2]) if len(sys.argv) > 2 else 8
rec = load_case(case)
bound, cbound, grids, params = load_scene(scene_of(case))
stage, wd = case_stage(case)
dec_b = {"coarse": cbound, "middle": bound, "fine": bound, "color": bound}
gt = rec["gt_depth"] if wd else None
args = (grids, params, dec_b, bound, rec["rays_o"], rec["rays_d"], stage, gt,
        (rec["g_depth"], rec["g_var"], rec["g_color"]))
truth = oracle_render_grads(*args, f64=True, round_inputs=True)
truth = {k: v for k, v in truth.items() if k in rec}
refs = [rec, oracle_render_grads_permuted(*args, seed=1), oracle_render_grads_permuted(*args, seed=2)]
worst = []
for seed in range(3, 3 + n_seeds):
    res = elementwise_vs_truth(oracle_render_grads_permuted(*args, seed=seed), refs, truth)
    k, v = max(res.items(), key=lambda kv: kv[1]["worst"])
    worst.append(v["worst"])
    print(f"[{case}] float32 permutation {seed}: worst ratio {v['worst']:.3f} ({k}, n_bad {v['n_bad']})", flush=True)
print(f"[{case}] {n_seeds} float32 implementations: worst ratio {min(worst):.3f} .. {max(worst):.3f}")
