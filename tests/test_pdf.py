"""Hierarchical sampling, sample_pdf (src/common.py:19-63; Renderer.py:244-250 when
N_importance > 0).

CPU: the oracle (oracle/pdf_oracle.py) against golden vectors produced by the
reference's own sample_pdf (tests/golden/make_golden_pdf.py): bit-exact.
GPU: nc_sample_pdf against the same vectors.  The float32 pdf normaliser is summed in
a different order than ATen's vectorised sum, so cdf entries may differ by an ulp:
samples agree within 1e-6 of the row's depth range plus 4 ulp of the cdf amplified by
1 / denom times the bin width (t = (u - cdf[below]) / denom), except where u lies within
4 ulp of a cdf entry -- there searchsorted's decision is a rounding tie (e.g. u = 1 against a
last cdf entry of 1 - 6e-8) and the sample may resolve into the neighbouring bin; such
samples must still lie inside that bin pair.  det and caller-drawn u, zero / one-hot /
peaked weights, one ray, the smallest bin count."""
import glob
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import pdf_oracle as PO

CASES = sorted(os.path.basename(p)[4:-4] for p in glob.glob(os.path.join(GOLDEN, "pdf_*.npz")))


def _load(name):
    z = np.load(os.path.join(GOLDEN, f"pdf_{name}.npz"))
    return {k: torch.from_numpy(z[k]) for k in z.files}


def test_golden_cases_present():
    assert len(CASES) >= 6


@pytest.mark.parametrize("name", CASES)
def test_oracle_matches_reference(name):
    g = _load(name)
    det = bool(g["det"])
    out = PO.sample_pdf(g["bins"], g["weights"], int(g["n_importance"]), det=det, u=None if det else g["u"])
    assert torch.equal(out, g["samples"])


def _ties(bins, weights, u, n):
    """Samples whose u lies within 4 ulp of an entry of the (reference-order) cdf."""
    w = weights + 1e-5
    cdf = torch.cumsum(w / w.sum(-1, keepdim=True), -1)
    cdf = torch.cat([torch.zeros_like(cdf[:, :1]), cdf], -1)
    if u is None:
        u = torch.linspace(0., 1., n).expand(cdf.shape[0], n)
    d = (u[:, :, None] - cdf[:, None, :]).abs()
    return (d <= 4 * 1.2e-7 * torch.clamp(u.abs(), min=1e-3)[:, :, None]).any(-1)


def _budget(bins, weights, u, n):
    """Per-sample error budget: a few float32 ulp of the cdf, amplified by 1 / denom
    (t = (u - cdf[below]) / denom), times the bin width, plus 1e-6 of the depth range."""
    w = weights + 1e-5
    cdf = torch.cumsum(w / w.sum(-1, keepdim=True), -1)
    cdf = torch.cat([torch.zeros_like(cdf[:, :1]), cdf], -1)
    if u is None:
        u = torch.linspace(0., 1., n).expand(cdf.shape[0], n).contiguous()
    inds = torch.searchsorted(cdf, u.contiguous(), right=True)
    below = (inds - 1).clamp(min=0)
    above = inds.clamp(max=cdf.shape[-1] - 1)
    c0, c1 = cdf.gather(1, below), cdf.gather(1, above)
    denom = torch.where(c1 - c0 < 1e-5, torch.ones_like(c0), c1 - c0)
    width = (bins.gather(1, above) - bins.gather(1, below)).abs()
    span = (bins[:, -1] - bins[:, 0]).abs()[:, None]
    return 1e-6 * span + (4 * 1.2e-7 / denom.double()) * width


def _assert_close(out, ref, bins, weights, u, n):
    err = (out - ref).abs()
    tie = _ties(bins, weights, u, n)
    bud = _budget(bins, weights, u, n)
    bad = (err > bud) & ~tie
    assert not bool(bad.any()), float((err / bud)[bad].max())
    assert bool((out >= bins[:, :1] - 1e-12).all() and (out <= bins[:, -1:] + 1e-12).all())
    # (ties: det's u = 0 against cdf[0] = 0 and u = 1 against the last entry, 1 +- ulp,
    # and, for uniform weights, u = k/(N-1) against cdf = j/(nb-1) exactly)


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_hip_matches_reference(name):
    from nicecore.ops import sample_pdf
    g = _load(name)
    det = bool(g["det"])
    out = sample_pdf(g["bins"].cuda(), g["weights"].cuda(), int(g["n_importance"]), det=det,
                     u=None if det else g["u"].cuda()).cpu()
    ref = g["samples"]
    _assert_close(out, ref, g["bins"], g["weights"], g["u"] if not det else None, int(g["n_importance"]))
    # monotone in u, inside the bins
    assert bool((out[:, 1:] >= out[:, :-1] - 1e-12).all()) if det else True
    assert bool((out >= g["bins"][:, :1] - 1e-12).all() and (out <= g["bins"][:, -1:] + 1e-12).all())


@pytest.mark.gpu
def test_hip_large_batch_against_oracle():
    """Renderer-sized batch (4096 rays, 48 samples -> 47 bins, 16 importance samples)."""
    from nicecore.ops import sample_pdf
    gen = torch.Generator().manual_seed(9)
    z = torch.sort(torch.rand(4096, 48, generator=gen, dtype=torch.float64) * 6 + 0.05, -1)[0]
    bins = 0.5 * (z[:, 1:] + z[:, :-1])
    w = (torch.rand(4096, 48, generator=gen) ** 4)[:, 1:-1].contiguous()
    u = torch.rand(4096, 16, generator=gen)
    for det in (True, False):
        ref = PO.sample_pdf(bins, w, 16, det=det, u=None if det else u)
        out = sample_pdf(bins.cuda(), w.cuda(), 16, det=det, u=None if det else u.cuda()).cpu()
        _assert_close(out, ref, bins, w, None if det else u, 16)


@pytest.mark.gpu
def test_hip_rejects_bad_shapes():
    from nicecore import _lib as L
    from nicecore.ops import sample_pdf
    b = torch.zeros(4, 70, dtype=torch.float64, device="cuda")
    with pytest.raises(L.NiceCoreError):
        sample_pdf(b, torch.zeros(4, 69, device="cuda"), 8, det=True)  # > 64 bins
    with pytest.raises(L.NiceCoreError):
        sample_pdf(b[:, :10], torch.zeros(4, 5, device="cuda"), 8, det=True)  # weights shape
