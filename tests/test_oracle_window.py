"""The oracle's windowed trilinear lookup (oracle/nice_oracle.py sample_grid_window) is the
checker the C5 parity tests use on windows of 26-GB grids that do not fit the CPU.  It
must compute what F.grid_sample (border, align_corners=True: decoder.py:179-188) computes
on the full grid: forward bit-identical, gradients to float rounding."""
import pytest
import torch
import torch.nn.functional as F

from oracle import nice_oracle as O


def _full(p, grid, bound):
    vg = O.normalize_3d_coordinate(p, bound).unsqueeze(0)[:, :, None, None].to(grid.dtype)
    c = F.grid_sample(grid, vg, padding_mode="border", align_corners=True, mode="bilinear")
    return c.squeeze(-1).squeeze(-1).transpose(1, 2).squeeze(0)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("window", [False, True])
def test_window_lookup_equals_grid_sample(dtype, window):
    gen = torch.Generator().manual_seed(4)
    D, H, W = 9, 11, 13
    grid = torch.randn(1, 32, D, H, W, generator=gen, dtype=dtype)
    bound = torch.tensor([[-1.0, 2.0], [0.5, 1.5], [-3.0, -1.0]], dtype=torch.float64)
    lo, hi = bound[:, 0], bound[:, 1]
    if window:  # points well inside a sub-box, window = their corners (+1 margin)
        u = 0.35 + 0.3 * torch.rand(3000, 3, generator=gen, dtype=torch.float64)
    else:  # whole grid incl. points outside the bound (border clipping) and on its faces
        u = -0.1 + 1.2 * torch.rand(3000, 3, generator=gen, dtype=torch.float64)
        u[:50] = torch.tensor([1.0, 0.0, 1.0], dtype=torch.float64)
    p = lo + (hi - lo) * u
    if window:
        idx = ((O.normalize_3d_coordinate(p, bound) + 1) / 2) * torch.tensor([W - 1, H - 1, D - 1])
        a = (idx.amin(0).floor() - 1).clamp_min(0).long()
        b = (idx.amax(0).ceil() + 1).long()
        x0, y0, z0 = a.tolist()
        x1, y1, z1 = b.tolist()
        sub = grid[:, :, z0:z1 + 1, y0:y1 + 1, x0:x1 + 1]
        assert sub.numel() < grid.numel()
        off = (z0, y0, x0)
    else:
        sub, off = grid, (0, 0, 0)
    p1 = p.clone().requires_grad_(True)
    g1 = grid.clone().requires_grad_(True)
    p2 = p.clone().requires_grad_(True)
    s2 = sub.clone().requires_grad_(True)
    old = O.FLOAT
    O.FLOAT = dtype
    try:
        ref = _full(p1, g1, bound)
        got = O.sample_grid_window(p2, s2, bound, (D, H, W), off)
    finally:
        O.FLOAT = old
    assert torch.equal(got, ref)
    up = torch.randn(ref.shape, generator=gen, dtype=dtype)
    ref.backward(up)
    got.backward(up)
    tol = 1e-5 if dtype == torch.float32 else 1e-12
    gref = g1.grad[:, :, off[0]:off[0] + sub.shape[2], off[1]:off[1] + sub.shape[3], off[2]:off[2] + sub.shape[4]]
    assert float((s2.grad - gref).abs().max()) <= tol * float(gref.abs().max())
    assert float(g1.grad.abs().sum()) == pytest.approx(float(gref.abs().sum()), rel=1e-9)  # nothing outside
    assert float((p2.grad - p1.grad).abs().max()) <= tol * float(p1.grad.abs().max())


def test_window_too_small_raises():
    grid = torch.zeros(1, 32, 5, 5, 5)
    bound = torch.tensor([[0.0, 1.0]] * 3, dtype=torch.float64)
    p = torch.full((4, 3), 0.5, dtype=torch.float64)
    with pytest.raises(ValueError):
        O.sample_grid_window(p, grid[:, :, :2, :2, :2], bound, (5, 5, 5), (0, 0, 0))
