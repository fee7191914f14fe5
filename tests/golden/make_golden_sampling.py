"""Golden vectors for the training-ray sampling (src/common.py:74-137) FROM THE
REFERENCE ITSELF.  Build container only (imports /root/reference's src.common).

For each case: seeded float32 / float64 poses, depth and colour images; the
reference's ``get_samples`` is called under ``torch.manual_seed(s)`` and the pixel
indices it drew are recovered by replaying ``torch.randint`` under the same seed
(select_uv's only random call, common.py:98).  A random upstream gradient is
back-propagated into c2w through the reference's rays.  Stored: inputs, indices,
outputs and d c2w.  Only numbers are written.

Usage:  python tests/golden/make_golden_sampling.py
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("NICE_REF", "/root/reference")

CASES = [
    # name, H, W, H0, H1, W0, W1, n, pose dtype, seed
    ("tracker_f32", 24, 32, 3, 21, 4, 28, 96, torch.float32, 1),
    ("mapper_f32", 24, 32, 0, 24, 0, 32, 128, torch.float32, 2),
    ("mapper_f64", 20, 36, 0, 20, 0, 36, 64, torch.float64, 3),
]
FX, FY, CX, CY = 30.0, 29.5, 15.5, 11.25


def random_pose(gen, dtype):
    q = torch.randn(4, generator=gen, dtype=torch.float64)
    q = q / q.norm()
    w, x, y, z = q.tolist()
    R = torch.tensor([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                      [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                      [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]], dtype=torch.float64)
    c2w = torch.eye(4, dtype=torch.float64)
    c2w[:3, :3] = R
    c2w[:3, 3] = torch.rand(3, generator=gen, dtype=torch.float64) * 2 - 1
    return c2w.to(dtype)


def main():
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    cwd = os.getcwd()
    os.chdir(REF)
    from src import common as ref_common
    os.chdir(cwd)
    for name, H, W, H0, H1, W0, W1, n, dtype, seed in CASES:
        gen = torch.Generator().manual_seed(100 + seed)
        c2w = random_pose(gen, dtype).requires_grad_(True)
        depth = torch.rand(H, W, generator=gen) * 4
        depth[torch.rand(H, W, generator=gen) < 0.1] = 0.0
        color = torch.rand(H, W, 3, generator=gen)
        torch.manual_seed(seed)
        ro, rd, d, c = ref_common.get_samples(H0, H1, W0, W1, n, H, W, FX, FY, CX, CY, c2w, depth, color, 'cpu')
        torch.manual_seed(seed)
        idx = torch.randint((H1 - H0) * (W1 - W0), (n,), device='cpu')
        g_o = torch.randn(ro.shape, generator=gen, dtype=ro.dtype)
        g_d = torch.randn(rd.shape, generator=gen, dtype=rd.dtype)
        torch.autograd.backward([ro, rd], [g_o, g_d])
        np.savez_compressed(os.path.join(HERE, f"sampling_{name}.npz"),
                            region=np.array([H0, H1, W0, W1]), intr=np.array([FX, FY, CX, CY]),
                            c2w=c2w.detach().numpy(), depth=depth.numpy(), color=color.numpy(),
                            indices=idx.numpy(), rays_o=ro.detach().numpy(), rays_d=rd.detach().numpy(),
                            gt_depth=d.numpy(), gt_color=c.numpy(), g_rays_o=g_o.numpy(),
                            g_rays_d=g_d.numpy(), grad_c2w=c2w.grad.numpy())
        print(name, ro.dtype, tuple(rd.shape), float(c2w.grad.abs().max()))


if __name__ == "__main__":
    main()
