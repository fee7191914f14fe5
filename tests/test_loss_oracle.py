"""The oracle's rendering losses (oracle/nice_oracle.py mapper_loss / tracker_loss,
restating Mapper.py:603-612 and Tracker.py:117-131) against a plain-Python loop
statement of the same definitions, on the golden render outputs.  The reference's
loss value itself is not held by any fixture ("parity unpinned" for the loss term,
DESIGN.md); these checks pin the oracle's semantics: the lower median, the masks,
the float32 colour term and the autograd derivatives the fused kernel reproduces."""
import math

import pytest
import torch

from conftest import load_case
from oracle import nice_oracle as O


def _lower_median(xs):
    if any(math.isnan(x) for x in xs):
        return math.nan
    return sorted(xs)[(len(xs) - 1) // 2]


def _loop_loss(kind, depth, var, color, gt, gtc, w, color_term, dyn):
    n = len(depth)
    tmp = [abs(float(gt[r]) - depth[r]) / math.sqrt(var[r] + 1e-10) for r in range(n)]
    if kind == "mapper":
        mask = [float(gt[r]) > 0 for r in range(n)]
        dsum = sum(abs(float(gt[r]) - depth[r]) for r in range(n) if mask[r])
        cmask = [True] * n
    else:
        thr = 10 * _lower_median(tmp) if dyn else math.inf
        mask = [float(gt[r]) > 0 and tmp[r] < thr for r in range(n)]
        dsum = sum(tmp[r] for r in range(n) if mask[r])
        cmask = mask
    csum = 0.0
    if color_term:
        csum = sum(abs(float(gtc[r][k]) - float(color[r][k])) for r in range(n) for k in range(3) if cmask[r])
    return dsum + w * csum, mask


@pytest.mark.parametrize("case", ["color_depth", "fine_depth", "middle_depth"])
@pytest.mark.parametrize("kind,color_term,dyn", [("mapper", False, False), ("mapper", True, False),
                                                 ("tracker", True, True), ("tracker", False, False),
                                                 ("tracker", False, True)])
def test_oracle_loss_matches_loop_statement(case, kind, color_term, dyn):
    rec = load_case(case)
    depth = rec["depth"].clone().requires_grad_(True)
    color = rec["color"].clone().requires_grad_(True)
    var, gt, gtc = rec["var"], rec["gt_depth"], rec["gt_color"]
    # make the dynamic mask bite: scale a few residuals up
    if dyn:
        with torch.no_grad():
            s = torch.sqrt(var + 1e-10)
            med = ((gt - depth).abs() / s).median()
            depth[::5] += 1000.0 * med * s[::5] + (gt - depth)[::5].abs()
    if kind == "mapper":
        L = O.mapper_loss(depth, color, gt, gtc, 0.2, color_term)
        w = 0.2
    else:
        L = O.tracker_loss(depth, var, color, gt, gtc, 0.5, color_term, dyn)
        w = 0.5
    ref, mask = _loop_loss(kind, depth.detach().tolist(), var.tolist(), color.detach().tolist(),
                           gt.tolist(), gtc.tolist(), w, color_term, dyn)
    assert L.dtype == torch.float64
    assert abs(float(L.detach()) - ref) <= 1e-6 * (abs(ref) + 1.0)
    if dyn:
        assert 0 < sum(mask) < sum(float(g) > 0 for g in gt.tolist())  # the outliers were dropped
    L.backward()
    # d loss / d depth: -sgn(gt - d) (/ sqrt(var + 1e-10) for the tracker) on masked rays
    for r in range(depth.shape[0]):
        diff = float(gt[r]) - float(depth.detach()[r])
        s = 1.0 if kind == "mapper" else math.sqrt(float(var[r]) + 1e-10)
        want = (-(1.0 if diff > 0 else -1.0 if diff < 0 else 0.0) / s) if mask[r] else 0.0
        assert abs(float(depth.grad[r]) - want) <= 1e-12 * max(1.0, abs(want))
    if color_term:
        assert color.grad is not None
        cm = torch.tensor(mask if kind == "tracker" else [True] * len(mask))
        want = -(w * torch.sign(gtc - color.detach())) * cm[:, None]
        assert torch.allclose(color.grad, want.float(), atol=1e-7)


def test_tracker_median_nan_drops_every_ray():
    """torch.median propagates NaN, so tmp < 10 * NaN masks every ray out."""
    d = torch.tensor([1.0, float("nan"), 2.0], dtype=torch.float64)
    v = torch.ones(3, dtype=torch.float64)
    gt = torch.tensor([1.5, 1.0, 1.0])
    L = O.tracker_loss(d, v, torch.zeros(3, 3), gt, None, 0.5, False, True)
    assert float(L) == 0.0
