"""ORACLE — TEST INFRASTRUCTURE ONLY.  Never imported by the product path.

CPU restatement of the reference's hierarchical (importance) sampling:

  sample_pdf   src/common.py:19-63   (NeRF §5.2 inverse-CDF sampling), called by
               Renderer.render_batch_ray when N_importance > 0 (Renderer.py:244-250)

The random draw (``torch.rand`` when det=False, common.py:36) is supplied as ``u``.
Parity status: PINNED against tests/golden/pdf_*.npz, produced by calling the
reference's own src.common.sample_pdf in the build container
(tests/golden/make_golden_pdf.py; det=False cases replay its torch.rand draw).
"""
from __future__ import annotations

import torch


def sample_pdf(bins, weights, N_samples, det=False, u=None):
    """common.py:19-63 with the uniform draw given as ``u`` when det is False."""
    weights = weights + 1e-5
    pdf = weights / torch.sum(weights, -1, keepdim=True)
    cdf = torch.cumsum(pdf, -1)
    cdf = torch.cat([torch.zeros_like(cdf[..., :1]), cdf], -1)
    if det:
        u = torch.linspace(0., 1., steps=N_samples)
        u = u.expand(list(cdf.shape[:-1]) + [N_samples])
    elif u is None:
        raise ValueError("det=False needs the uniform draw u")
    u = u.contiguous()
    inds = torch.searchsorted(cdf, u, right=True)
    below = torch.max(torch.zeros_like(inds - 1), inds - 1)
    above = torch.min((cdf.shape[-1] - 1) * torch.ones_like(inds), inds)
    inds_g = torch.stack([below, above], -1)
    matched_shape = [inds_g.shape[0], inds_g.shape[1], cdf.shape[-1]]
    cdf_g = torch.gather(cdf.unsqueeze(1).expand(matched_shape), 2, inds_g)
    bins_g = torch.gather(bins.unsqueeze(1).expand(matched_shape), 2, inds_g)
    denom = cdf_g[..., 1] - cdf_g[..., 0]
    denom = torch.where(denom < 1e-5, torch.ones_like(denom), denom)
    t = (u - cdf_g[..., 0]) / denom
    return bins_g[..., 0] + t * (bins_g[..., 1] - bins_g[..., 0])
