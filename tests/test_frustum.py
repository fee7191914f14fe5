"""Frustum feature selection: the numpy oracle's cv2.remap
restatement on hand-checked cases (CPU), and the HIP kernels against the oracle on
Replica room0-sized grids (GPU).

Parity: UNPINNED against the reference (cv2 is absent here, oracle/frustum_oracle.py).
The mask is a threshold decision on float results that the reference computes with
numpy/OpenBLAS matmuls; the kernel uses the same operations and dtypes but not the
same BLAS summation order, so a voxel whose decision margin is below 1e-4 (pixels /
metres) may flip.  Bar: no disagreement with a margin above that, and at most
1e-4 of the voxels disagreeing at all."""
import numpy as np
import pytest
import torch

from oracle import frustum_oracle as FO


def test_remap_restatement_known_values():
    img = np.arange(12, dtype=np.float32).reshape(3, 4)
    x = np.array([0.0, 1.0, 0.5, 2.25, 3.0, 3.5, -0.5, -1.5, 1.0, 10.0], dtype=np.float32)
    y = np.array([0.0, 2.0, 0.0, 1.0, 2.0, 0.0, 0.0, 0.0, 0.5, 0.0], dtype=np.float32)
    d = FO.cv2_remap_linear(img, x, y)
    # exact taps; half pixel = mean; 1/4 pixel; last column (x+1 tap is border 0);
    # half outside (left tap 0); fully outside -> 0; vertical half
    np.testing.assert_array_equal(d[:2], [0.0, 9.0])
    assert d[2] == 0.5 and d[3] == 6.25 and d[4] == 11.0
    assert d[5] == 1.5 and d[6] == 0.0 and d[7] == 0.0
    assert d[8] == 3.0 and d[9] == 0.0
    # 5-bit sub-pixel quantisation with round-half-even: 1/64 rounds to 0, 3/64 to 2/32
    q = FO.cv2_remap_linear(img, np.array([1 / 64, 3 / 64], np.float32), np.zeros(2, np.float32))
    assert q[0] == 0.0 and q[1] == np.float32(2 / 32)


def _room0_frame(seed):
    from nicecore import scene as S
    sc = S.make_scene("replica_room0")
    gen = torch.Generator().manual_seed(seed)
    # camera inside the room looking along a random direction
    q = torch.randn(4, generator=gen, dtype=torch.float64)
    q = q / q.norm()
    w, x, y, z = q.tolist()
    R = torch.tensor([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                      [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                      [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])
    b = sc.bound
    t = b[:, 0] + (b[:, 1] - b[:, 0]) * (0.3 + 0.4 * torch.rand(3, generator=gen, dtype=torch.float64))
    c2w = torch.eye(4)
    c2w[:3, :3] = R.float()
    c2w[:3, 3] = t.float()
    depth = (torch.rand(sc.H, sc.W, generator=gen) * 4 + 0.5)
    depth[torch.rand(sc.H, sc.W, generator=gen) < 0.05] = 0.0
    return sc, c2w, depth.numpy()


@pytest.mark.gpu
@pytest.mark.parametrize("key", ["grid_middle", "grid_fine", "grid_coarse"])
@pytest.mark.parametrize("seed", [1, 2])
def test_frustum_mask_matches_oracle(key, seed):
    from nicecore.frustum import FrustumSelector
    sc, c2w, depth = _room0_frame(seed)
    shape = sc.shapes[key][-3:]
    bound = sc.bound if key != "grid_coarse" else sc.bound * 2
    sel = FrustumSelector(bound, sc.H, sc.W, sc.fx, sc.fy, sc.cx, sc.cy)
    got = sel.get_mask_from_c2w(c2w, key, shape, depth).cpu().numpy()
    ref = FO.get_mask_from_c2w(c2w, key, shape, depth, bound, sc.H, sc.W, sc.fx, sc.fy, sc.cx, sc.cy)
    assert got.shape == ref.shape
    if key == "grid_coarse":
        assert got.all()
        return
    assert 0 < ref.sum() < ref.size  # the frame sees part of the grid
    diff = got != ref
    if diff.any():
        m = FO.margins(c2w, shape, depth, bound, sc.H, sc.W, sc.fx, sc.fy, sc.cx, sc.cy)
        assert float(m[diff].max()) < 1e-4, float(m[diff].max())
        assert diff.mean() <= 1e-4, diff.mean()
    # the Mapper's use: permute(2,1,0) gives the grid-order mask
    g = sel.grid_mask(c2w, key, shape, depth)
    assert torch.equal(g.cpu(), torch.from_numpy(got).permute(2, 1, 0).contiguous())
