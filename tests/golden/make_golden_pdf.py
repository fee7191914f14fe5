"""Golden vectors for hierarchical sampling, sample_pdf (src/common.py:19-63), FROM THE
REFERENCE ITSELF.  Build container only (imports /root/reference's src.common).

Inputs are shaped as Renderer.render_batch_ray passes them when N_importance > 0
(Renderer.py:244-250): bins = the mid-points of sorted float64 sample depths, weights =
float32 compositing weights without the first and last sample.  det=False cases
replay the reference's torch.rand draw under the same seed to store u.  Edge cases:
all-zero weights, one-hot weights, a single ray, the smallest bin count.  Only
numbers are written.

Usage:  python tests/golden/make_golden_pdf.py
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("NICE_REF", "/root/reference")

CASES = [
    # name, rays, samples per ray (z), N_importance, det, seed, weights kind
    ("imap_det", 64, 32, 12, True, 1, "random"),
    ("rand", 48, 48, 16, False, 2, "random"),
    ("peaked_det", 32, 40, 24, True, 3, "peaked"),
    ("zero_weights_det", 8, 16, 8, True, 4, "zero"),
    ("onehot_rand", 16, 20, 10, False, 5, "onehot"),
    ("one_ray_small", 1, 3, 5, True, 6, "random"),
]


def make_inputs(n, s, kind, gen):
    z = torch.sort(torch.rand(n, s, generator=gen, dtype=torch.float64) * 5 + 0.1, -1)[0]
    bins = 0.5 * (z[..., 1:] + z[..., :-1])
    if kind == "random":
        w = torch.rand(n, s, generator=gen) ** 3
    elif kind == "peaked":
        c = torch.randint(0, s, (n, 1), generator=gen).float()
        w = torch.exp(-0.5 * ((torch.arange(s).float() - c) / 1.5) ** 2)
    elif kind == "zero":
        w = torch.zeros(n, s)
    else:
        w = torch.zeros(n, s)
        w[torch.arange(n), torch.randint(1, s - 1, (n,), generator=gen)] = 1.0
    return bins, w[..., 1:-1].contiguous()


def main():
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    cwd = os.getcwd()
    os.chdir(REF)
    from src import common as ref_common
    os.chdir(cwd)
    for name, n, s, nimp, det, seed, kind in CASES:
        gen = torch.Generator().manual_seed(200 + seed)
        bins, w = make_inputs(n, s, kind, gen)
        torch.manual_seed(seed)
        out = ref_common.sample_pdf(bins, w, nimp, det=det, device='cpu')
        torch.manual_seed(seed)
        u = torch.rand(n, nimp) if not det else torch.linspace(0., 1., nimp).expand(n, nimp)
        np.savez_compressed(os.path.join(HERE, f"pdf_{name}.npz"), bins=bins.numpy(), weights=w.numpy(),
                            u=u.contiguous().numpy(), det=np.array(det), n_importance=np.array(nimp),
                            samples=out.numpy())
        print(name, tuple(out.shape), out.dtype)


if __name__ == "__main__":
    main()
