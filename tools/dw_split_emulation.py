"""Diagnostic (CPU): can k_mlp_dw run on the split-f16 MFMA with ONE power-of-two scale per
job and operand side?  The float32 oracle with every linear layer's weight gradient
computed from operands rounded as such a kernel would (x s = hi + lo, two round-to-nearest
f16 halves, s = 2^(14 - exponent(max |x|)) over the whole tensor; float32 accumulation),
scored with the per-element gate of tests/test_gpu_elementwise.py against plain float32 dW.
    python tools/dw_split_emulation.py [case ...]"""
import os, sys, torch
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "nice-slam-annotation_amd"), os.path.join(REPO, "tests")):
    sys.path.insert(0, p)
from conftest import load_case, load_scene, CASE_NAMES, INITSTD_CASES
from parity_common import case_stage, elementwise_vs_truth, oracle_render_grads, oracle_render_grads_permuted, scene_of
from oracle import nice_oracle as O
import torch.nn.functional as F

def split(x):  # job-wide power-of-two scale: max at 2^14
    m = float(x.abs().max())
    if m == 0: return x
    e = torch.floor(torch.log2(torch.tensor(m)))
    s = float(2.0 ** (14 - e))
    xs = x * s
    hi = xs.half().float()
    lo = (xs - hi).half().float()
    return (hi + lo) / s

class Lin(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        return F.linear(x, w, b)
    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        gx = gy @ w
        gw = (split(gy).t() @ split(x)) if MODE else gy.t() @ x
        return gx, gw, gy.sum(0)

_lin0 = O._lin
def _lin(x, prm, name):
    if x.dtype != torch.float32: return _lin0(x, prm, name)
    return Lin.apply(x, prm[name + '.weight'], prm[name + '.bias'])

cases = sys.argv[1:] or (CASE_NAMES + INITSTD_CASES)
for case in cases:
    rec = load_case(case)
    bound, cbound, grids, params = load_scene(scene_of(case))
    stage, wd = case_stage(case)
    dec_b = {"coarse": cbound, "middle": bound, "fine": bound, "color": bound}
    gt = rec["gt_depth"] if wd else None
    args = (grids, params, dec_b, bound, rec["rays_o"], rec["rays_d"], stage, gt, (rec["g_depth"], rec["g_var"], rec["g_color"]))
    truth = oracle_render_grads(*args, f64=True, round_inputs=True)
    truth = {k: v for k, v in truth.items() if k in rec}
    refs = [rec, oracle_render_grads_permuted(*args, seed=1), oracle_render_grads_permuted(*args, seed=2)]
    O._lin = _lin
    out = {}
    for MODE in (0, 1):
        got = oracle_render_grads(*args)
        res = elementwise_vs_truth(got, refs, truth)
        k, v = max(((k, v) for k, v in res.items() if "weight" in k or "_B" in k), key=lambda kv: kv[1]["worst"])
        out[MODE] = (round(v["worst"], 3), k.split("/")[-1])
    O._lin = _lin0
    print(case, "plain f32 dW:", out[0], " split dW:", out[1], flush=True)
