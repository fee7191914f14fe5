"""Training-ray sampling: the oracle against golden vectors from
the reference's src.common.get_samples (CPU), and the HIP kernels (nc_sample.hip,
through the C ABI) against both.

Tolerances: rays, gathered depth / colour and the pre-filter mask bit-exact (same
float32 / float64 operations in the same order); d c2w (a sum over the frame's rays,
tree order on the GPU vs torch's reduction) <= 1e-6 of max-abs in float32,
1e-12 in float64."""
import glob
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import sampling_oracle as SO

CASES = sorted(os.path.basename(p)[len("sampling_"):-4] for p in glob.glob(os.path.join(GOLDEN, "sampling_*.npz")))


def load(name):
    z = np.load(os.path.join(GOLDEN, f"sampling_{name}.npz"))
    return {k: torch.from_numpy(z[k]) for k in z.files}


def rel(a, b):
    a, b = a.double().reshape(-1), b.double().reshape(-1)
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def test_golden_cases_present():
    assert {"tracker_f32", "mapper_f32", "mapper_f64"} <= set(CASES)


@pytest.mark.parametrize("name", CASES)
def test_oracle_matches_reference(name):
    z = load(name)
    H0, H1, W0, W1 = z["region"].tolist()
    fx, fy, cx, cy = z["intr"].tolist()
    c2w = z["c2w"].clone().requires_grad_(True)
    ro, rd, d, c = SO.get_samples(H0, H1, W0, W1, z["indices"], fx, fy, cx, cy, c2w, z["depth"], z["color"])
    assert torch.equal(ro.detach(), z["rays_o"]) and torch.equal(rd.detach(), z["rays_d"])
    assert torch.equal(d, z["gt_depth"]) and torch.equal(c, z["gt_color"])
    torch.autograd.backward([ro, rd], [z["g_rays_o"], z["g_rays_d"]])
    torch.testing.assert_close(c2w.grad, z["grad_c2w"], rtol=0, atol=0)


def test_bbox_mask_semantics():
    """NaN (0/0 on an axis) -> outside; t is the exit distance of the box."""
    bound = torch.tensor([[-1.0, 1.0], [-1.0, 1.0], [-1.0, 1.0]], dtype=torch.float64)
    o = torch.tensor([[0.0, 0.0, 0.0], [0.0, 0.0, 0.0], [1.0, 0.0, 0.0]])
    d = torch.tensor([[1.0, 0.5, 0.25], [1.0, 0.5, 0.25], [0.0, 1.0, 1.0]])
    gt = torch.tensor([0.9, 1.1, 0.1])
    m = SO.bbox_inside_mask(bound, o, d, gt)
    assert m.tolist() == [True, False, False]


def _gpu_case(name, bound=None):
    from nicecore import sampling as NS
    z = load(name)
    H0, H1, W0, W1 = z["region"].tolist()
    fx, fy, cx, cy = z["intr"].tolist()
    c2w = z["c2w"].cuda().requires_grad_(True)
    out = NS.sample_frames(H0, H1, W0, W1, z["indices"].shape[0], fx, fy, cx, cy, c2w[None],
                           z["depth"].cuda()[None], z["color"].cuda()[None], bound=bound,
                           indices=z["indices"].cuda()[None])
    return z, c2w, out


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_hip_matches_reference(name):
    z, c2w, (ro, rd, d, c, inside) = _gpu_case(name)
    assert ro.dtype == z["rays_o"].dtype
    assert torch.equal(ro.detach().cpu(), z["rays_o"]) and torch.equal(rd.detach().cpu(), z["rays_d"])
    assert torch.equal(d.cpu(), z["gt_depth"]) and torch.equal(c.cpu(), z["gt_color"])
    assert inside is None
    torch.autograd.backward([ro, rd], [z["g_rays_o"].cuda(), z["g_rays_d"].cuda()])
    tol = 1e-12 if c2w.dtype == torch.float64 else 1e-6
    assert c2w.grad.shape == (4, 4)
    assert rel(c2w.grad.cpu(), z["grad_c2w"]) <= tol
    assert float(c2w.grad[3].abs().max()) == 0.0


@pytest.mark.gpu
def test_hip_drop_in_get_samples_and_uv():
    """get_samples / get_rays_from_uv with the reference's signatures; the RNG draw is
    select_uv's (same pixels under the same seed)."""
    from nicecore import sampling as NS
    z = load("tracker_f32")
    H0, H1, W0, W1 = z["region"].tolist()
    fx, fy, cx, cy = z["intr"].tolist()
    H, W = z["depth"].shape
    n = z["indices"].shape[0]
    dev = "cuda"
    torch.manual_seed(5)
    ro, rd, d, c = NS.get_samples(H0, H1, W0, W1, n, H, W, fx, fy, cx, cy, z["c2w"].cuda(),
                                  z["depth"].cuda(), z["color"].cuda(), dev)
    torch.manual_seed(5)
    idx = torch.randint((H1 - H0) * (W1 - W0), (n,), device=dev).cpu()
    ro_o, rd_o, d_o, c_o = SO.get_samples(H0, H1, W0, W1, idx, fx, fy, cx, cy, z["c2w"], z["depth"], z["color"])
    assert torch.equal(rd.cpu(), rd_o) and torch.equal(ro.cpu(), ro_o)
    assert torch.equal(d.cpu(), d_o) and torch.equal(c.cpu(), c_o)
    # caller uv (fractional pixels too)
    gen = torch.Generator().manual_seed(9)
    i = torch.rand(50, generator=gen) * W
    j = torch.rand(50, generator=gen) * H
    ro2, rd2 = NS.get_rays_from_uv(i.cuda(), j.cuda(), z["c2w"].cuda(), H, W, fx, fy, cx, cy, dev)
    ro3, rd3 = SO.get_rays_from_uv(i, j, z["c2w"], fx, fy, cx, cy)
    assert torch.equal(rd2.cpu(), rd3) and torch.equal(ro2.cpu(), ro3)


@pytest.mark.gpu
def test_hip_frames_batch_and_prefilter():
    """Mapper-style batch: F poses (some requiring grad), images from a resident stack
    picked by frame_ids, bbox pre-filter mask; against the oracle's per-frame loop."""
    from nicecore import sampling as NS
    gen = torch.Generator().manual_seed(3)
    K, F, H, W, n = 6, 4, 30, 40, 200
    fx, fy, cx, cy = 35.0, 35.0, 19.5, 14.5
    depths = torch.rand(K, H, W, generator=gen) * 3
    depths[torch.rand(K, H, W, generator=gen) < 0.1] = 0
    colors = torch.rand(K, H, W, 3, generator=gen)
    fid = torch.tensor([5, 0, 3, 3])
    c2ws = []
    for f in range(F):
        q = torch.randn(4, generator=gen, dtype=torch.float64)
        q = q / q.norm()
        w, x, y, zq = q.tolist()
        R = torch.tensor([[1 - 2 * (y * y + zq * zq), 2 * (x * y - zq * w), 2 * (x * zq + y * w)],
                          [2 * (x * y + zq * w), 1 - 2 * (x * x + zq * zq), 2 * (y * zq - x * w)],
                          [2 * (x * zq - y * w), 2 * (y * zq + x * w), 1 - 2 * (x * x + y * y)]])
        t = torch.rand(3, 1, generator=gen) - 0.5
        c2ws.append(torch.cat([R.float(), t], 1))
    c2w = torch.stack(c2ws)
    bound = torch.tensor([[-1.5, 1.5], [-1.2, 1.2], [-2.0, 2.0]], dtype=torch.float64)
    idx = torch.randint(H * W, (F, n), generator=gen)
    # oracle
    c2w_o = c2w.clone().requires_grad_(True)
    ro_o, rd_o, d_o, c_o, in_o = SO.frames(0, H, 0, W, idx, fx, fy, cx, cy, list(c2w_o),
                                           [depths[k] for k in fid], [colors[k] for k in fid], bound)
    # HIP
    c2w_g = c2w.cuda().requires_grad_(True)
    ro, rd, d, c, inside = NS.sample_frames(0, H, 0, W, n, fx, fy, cx, cy, c2w_g, depths.cuda(), colors.cuda(),
                                            frame_ids=fid.cuda(), bound=bound, indices=idx.cuda())
    assert torch.equal(ro.detach().cpu(), ro_o.detach()) and torch.equal(rd.detach().cpu(), rd_o.detach())
    assert torch.equal(d.cpu(), d_o) and torch.equal(c.cpu(), c_o)
    assert torch.equal(inside.cpu(), in_o) and 0 < int(in_o.sum()) < F * n
    # gradient through the compacted batch, as the callers use it
    gen2 = torch.Generator().manual_seed(4)
    m = in_o
    wo = torch.randn(int(m.sum()), 3, generator=gen2)
    wd = torch.randn(int(m.sum()), 3, generator=gen2)
    ((ro_o[m] * wo).sum() + (rd_o[m] * wd).sum()).backward()
    ro_c, rd_c, _, _ = NS.bbox_filter(ro, rd, d, c, inside)
    ((ro_c * wo.cuda()).sum() + (rd_c * wd.cuda()).sum()).backward()
    assert rel(c2w_g.grad.cpu(), c2w_o.grad) <= 1e-5



@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_hip_camera_tensor_sampling(dtype):
    """sample_frames_from_tensor (ABI v11): get_camera_from_tensor (common.py:163-176) inside
    the sampling kernel and its backward inside the pose-gradient kernel, against the
    reference's torch ops (oracle.sampling_oracle.camera_from_tensor) feeding sample_frames:
    rays to float rounding, the camera-tensor gradient to 1e-5 of max-abs -- with quaternions
    off unit norm (two_s = 2 / |q|^2), as Adam leaves them, and several frames."""
    from nicecore import sampling as NS
    gen = torch.Generator().manual_seed(21)
    K, F, H, W, n = 3, 3, 30, 40, 300
    fx, fy, cx, cy = 35.0, 35.0, 19.5, 14.5
    depths = (torch.rand(K, H, W, generator=gen) * 3).cuda()
    colors = torch.rand(K, H, W, 3, generator=gen).cuda()
    cam = torch.cat([torch.randn(F, 4, generator=gen) * 0.7, torch.rand(F, 3, generator=gen) - 0.5], 1).to(dtype)
    bound = torch.tensor([[-1.5, 1.5], [-1.2, 1.2], [-2.0, 2.0]], dtype=torch.float64)
    idx = torch.randint(H * W, (F, n), generator=gen).cuda()
    fid = torch.tensor([2, 0, 1]).cuda()
    up_o, up_d = (torch.randn(F * n, 3, generator=gen, dtype=dtype).cuda() for _ in range(2))
    # the reference's ops
    c1 = cam.cuda().requires_grad_(True)
    ro1, rd1, d1, col1, in1 = NS.sample_frames(0, H, 0, W, n, fx, fy, cx, cy, SO.camera_from_tensor(c1), depths,
                                               colors, frame_ids=fid, bound=bound, indices=idx)
    ((ro1 * up_o).sum() + (rd1 * up_d).sum()).backward()
    # fused
    c2 = cam.cuda().requires_grad_(True)
    ro2, rd2, d2, col2, in2 = NS.sample_frames_from_tensor(0, H, 0, W, n, fx, fy, cx, cy, c2, depths, colors,
                                                           frame_ids=fid, bound=bound, indices=idx)
    ((ro2 * up_o).sum() + (rd2 * up_d).sum()).backward()
    tol = 1e-6 if dtype == torch.float32 else 1e-13
    assert rel(ro2.detach().cpu(), ro1.detach().cpu()) <= tol and rel(rd2.detach().cpu(), rd1.detach().cpu()) <= tol
    assert torch.equal(d1, d2) and torch.equal(col1, col2)
    assert int((in1 != in2).sum()) <= 1  # a ray exactly on the filter's edge may flip with the last bit
    assert rel(c2.grad.cpu(), c1.grad.cpu()) <= (1e-5 if dtype == torch.float32 else 1e-12)
    # one camera as a [7] tensor, the Tracker's form
    c3 = cam[0].cuda().requires_grad_(True)
    ro3, rd3, _, _, _ = NS.sample_frames_from_tensor(0, H, 0, W, n, fx, fy, cx, cy, c3, depths, colors,
                                                     indices=idx[:1])
    (rd3.sum() + ro3.sum()).backward()
    assert c3.grad.shape == (7,) and bool(torch.isfinite(c3.grad).all())


def test_oracle_camera_tensor_rotation_is_float32():
    """common.py:150: quad2rotation assigns R into torch.zeros(bs, 3, 3) -- float32 whatever
    the quaternion's dtype -- and get_camera_from_tensor's cat promotes it (common.py:173):
    a float64 camera tensor gives float32-rounded rotation entries and a float64
    translation, and R's gradient is rounded to float32 on its way to the quaternion."""
    gen = torch.Generator().manual_seed(3)
    cam = torch.cat([torch.randn(2, 4, generator=gen, dtype=torch.float64),
                     torch.randn(2, 3, generator=gen, dtype=torch.float64)], 1).requires_grad_(True)
    RT = SO.camera_from_tensor(cam)
    assert RT.dtype == torch.float64
    R = RT[:, :, :3].detach()
    assert torch.equal(R, R.float().double())  # float32-representable
    assert torch.equal(RT[:, :, 3].detach(), cam[:, 4:].detach())  # translation untouched
    g = torch.randn(RT.shape, generator=gen, dtype=torch.float64)
    (RT * g).sum().backward()
    # the same chain with the upstream rotation gradient rounded to float32 by hand
    q = cam.detach()[:, :4].clone().requires_grad_(True)
    R64 = SO.quad2rotation(q)
    (R64.double() * g[:, :, :3].float().double()).sum().backward()
    assert torch.equal(cam.grad[:, :4], q.grad)
