"""The CPU oracle (oracle/nice_oracle.py) against golden vectors captured from the
reference renderer (tests/golden/make_golden.py).  Pins the oracle."""
import pytest
import torch

from conftest import CASE_NAMES, load_case, load_meta, load_scene
from oracle import nice_oracle as O


def _run(case, grids_req=True):
    meta = load_meta()
    stage = next(c for c in meta["cases"] if c["name"] == case)["stage"]
    bound, cbound, grids, params = load_scene()
    rec = load_case(case)
    ro = rec["rays_o"].clone().requires_grad_(True)
    rd = rec["rays_d"].clone().requires_grad_(True)
    g = {k: v.clone().requires_grad_(grids_req) for k, v in grids.items()}
    prm = {k: v.clone().requires_grad_(True) for k, v in params.items()}
    with_depth = next(c for c in meta["cases"] if c["name"] == case)["with_depth"]
    gt = rec["gt_depth"] if with_depth else None
    dec_bounds = {"coarse": cbound, "middle": bound, "fine": bound, "color": bound}
    depth, var, color = O.render_batch_ray(g, prm, dec_bounds, bound, rd, ro, stage, gt,
                                           meta["n_samples"], meta["n_surface"])
    torch.autograd.backward([depth, var, color], [rec["g_depth"], rec["g_var"], rec["g_color"]])
    return rec, (depth, var, color), ro, rd, g, prm, stage, bound, dec_bounds, gt


@pytest.mark.parametrize("case", CASE_NAMES)
def test_oracle_outputs_and_grads(case):
    rec, (depth, var, color), ro, rd, g, prm, *_ = _run(case)
    # same torch CPU ops, same order -> bitwise or last-ulp equal
    torch.testing.assert_close(depth.detach(), rec["depth"], rtol=1e-12, atol=1e-13)
    torch.testing.assert_close(var.detach(), rec["var"], rtol=1e-12, atol=1e-13)
    torch.testing.assert_close(color.detach(), rec["color"], rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(ro.grad, rec["grad/rays_o"], rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(rd.grad, rec["grad/rays_d"], rtol=1e-5, atol=1e-6)
    for k, v in g.items():
        key = "grad/" + k
        if key in rec:
            torch.testing.assert_close(v.grad, rec[key], rtol=1e-5, atol=1e-7)
        else:
            assert v.grad is None or float(v.grad.abs().max()) == 0.0
    for k, v in prm.items():
        key = "grad/param/" + k
        if key in rec:
            torch.testing.assert_close(v.grad, rec[key], rtol=1e-5, atol=1e-6)
        else:
            assert v.grad is None or float(v.grad.abs().max()) == 0.0


@pytest.mark.parametrize("case", CASE_NAMES)
def test_oracle_sample_points_and_raw(case):
    meta = load_meta()
    rec, _, ro, rd, g, prm, stage, bound, dec_bounds, gt = _run(case)
    z, pts = O.points_for_rays(rec["rays_o"], rec["rays_d"], bound, gt, stage,
                               meta["n_samples"], meta["n_surface"])
    assert torch.equal(pts.reshape(-1, 3), rec["pts"])  # float64 chain is exact
    with torch.no_grad():
        raw = O.eval_points(rec["pts"], {k: v.detach() for k, v in g.items()},
                            {k: v.detach() for k, v in prm.items()}, bound, dec_bounds, stage)
    torch.testing.assert_close(raw, rec["raw"], rtol=0, atol=0)


# ---- C1 = BASELINE configs[0] (tests/golden/make_golden_c1.py) ----
from parity_common import C1_CASES, c1_inputs  # noqa: E402


@pytest.mark.parametrize("case", [c[0] for c in C1_CASES])
def test_oracle_c1_golden(case):
    """Replica room0, 200 rays x 32 samples, stage middle: the oracle (float32, the
    reference's op order) on the regenerated grids / parameters against the reference's
    own outputs and gradients at BASELINE's configs[0]."""
    sc, grids, params, (ro0, rd0) = c1_inputs(case)
    rec = load_case(case)
    assert torch.equal(ro0, rec["rays_o"]) and torch.equal(rd0, rec["rays_d"])  # same rays regenerated
    ro = rec["rays_o"].clone().requires_grad_(True)
    rd = rec["rays_d"].clone().requires_grad_(True)
    g = {k: v.clone().requires_grad_(True) for k, v in grids.items()}
    prm = {k: v.clone().requires_grad_(True) for k, v in params.items()}
    dec_bounds = {"coarse": sc.bound * 2, "middle": sc.bound, "fine": sc.bound, "color": sc.bound}
    depth, var, color = O.render_batch_ray(g, prm, dec_bounds, sc.bound, rd, ro, "middle", None)
    torch.autograd.backward([depth, var, color], [rec["g_depth"], rec["g_var"], rec["g_color"]])
    torch.testing.assert_close(depth.detach(), rec["depth"], rtol=1e-12, atol=1e-13)
    torch.testing.assert_close(var.detach(), rec["var"], rtol=1e-12, atol=1e-13)
    torch.testing.assert_close(color.detach(), rec["color"], rtol=0, atol=0)
    torch.testing.assert_close(ro.grad, rec["grad/rays_o"], rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(rd.grad, rec["grad/rays_d"], rtol=1e-5, atol=1e-6)
    gm = rec["grad/grid_middle"]
    torch.testing.assert_close(g["grid_middle"].grad, gm, rtol=1e-5, atol=1e-6 * float(gm.abs().max()))
    for k in ("grid_coarse", "grid_fine", "grid_color"):
        assert g[k].grad is None or float(g[k].grad.abs().max()) == 0.0
    for k, v in prm.items():
        key = "grad/param/" + k
        if key in rec:
            torch.testing.assert_close(v.grad, rec[key], rtol=1e-5, atol=1e-6 * float(rec[key].abs().max()))
        else:
            assert v.grad is None or float(v.grad.abs().max()) == 0.0


# ---- iMAP* (tests/golden/make_golden_imap.py) ----
import json  # noqa: E402
import os  # noqa: E402

import numpy as np  # noqa: E402

from oracle import imap_oracle as IO  # noqa: E402

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
IMAP_META = json.load(open(os.path.join(GOLD, "imap_meta.json")))
IMAP_CASES = [c["name"] for c in IMAP_META["cases"]]


def load_imap(name):
    with np.load(os.path.join(GOLD, f"imap_{name}.npz")) as z:
        return {k: torch.from_numpy(z[k]) for k in z.files}


def imap_scene():
    with np.load(os.path.join(GOLD, "imap_scene.npz")) as z:
        d = {k: torch.from_numpy(z[k]) for k in z.files}
    return d["bound"], {k[len("param/"):]: v for k, v in d.items() if k.startswith("param/")}


def run_imap_oracle(name):
    case = next(c for c in IMAP_META["cases"] if c["name"] == name)
    bound, params = imap_scene()
    rec = load_imap(name)
    ro = rec["rays_o"].clone().requires_grad_(True)
    rd = rec["rays_d"].clone().requires_grad_(True)
    prm = {k: v.clone().requires_grad_(True) for k, v in params.items()}
    gt = rec["gt_depth"] if case["with_depth"] else None
    out = IO.render_batch_ray(prm, bound, rd, ro, gt, IMAP_META["n_samples"], case["n_importance"])
    torch.autograd.backward(list(out), [rec["g_depth"], rec["g_var"], rec["g_color"]])
    return rec, out, ro, rd, prm, bound


@pytest.mark.parametrize("case", IMAP_CASES)
def test_imap_oracle_outputs_and_grads(case):
    rec, (depth, var, color), ro, rd, prm, bound = run_imap_oracle(case)
    torch.testing.assert_close(depth.detach(), rec["depth"], rtol=1e-12, atol=1e-13)
    torch.testing.assert_close(var.detach(), rec["var"], rtol=1e-12, atol=1e-13)
    torch.testing.assert_close(color.detach(), rec["color"], rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(ro.grad, rec["grad/rays_o"], rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(rd.grad, rec["grad/rays_d"], rtol=1e-5, atol=1e-6)
    for k, v in prm.items():
        torch.testing.assert_close(v.grad, rec["grad/param/" + k], rtol=1e-5, atol=1e-6)
    with torch.no_grad():
        raw = IO.eval_points(rec["pts"], {k: v.detach() for k, v in prm.items()}, bound)
    torch.testing.assert_close(raw, rec["raw"], rtol=0, atol=0)
