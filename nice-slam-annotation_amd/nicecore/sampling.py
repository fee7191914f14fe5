"""Training-ray sampling on the HIP core (ABI v4, nc_sample_rays_*).

Drop-ins for the reference's helpers (same names, arguments and return values):

  get_rays_from_uv(i, j, c2w, H, W, fx, fy, cx, cy, device)        src/common.py:74-89
  get_samples(H0, H1, W0, W1, n, H, W, fx, fy, cx, cy, c2w, depth, color, device)
                                                                    src/common.py:126-137

plus the batched form the Mapper's per-keyframe loop (Mapper.py:543-591) and the
Tracker (Tracker.py:95-111) amount to:

  sample_frames(H0, H1, W0, W1, n, fx, fy, cx, cy, c2w[F], depth[K], color[K],
                frame_ids=None, bound=None, indices=None)
      -> rays_o, rays_d, gt_depth, gt_color, inside

one launch over all frames, reading the depth / colour images from a resident
keyframe stack (``frame_ids`` picks each pose's image; no per-iteration host-to-device
image copies), with the bbox pre-filter mask computed in the same pass.  The pose
gradient (rays -> c2w) is one more launch; ``get_camera_from_tensor`` (quaternion ->
R, t) stays a few torch ops upstream of it, so camera tensors get their gradient
through ordinary autograd.

Pixel draws: ``torch.randint(region_size, (n,), device=device)`` per frame, exactly
select_uv's call (common.py:98), so under the same RNG state the same pixels are
chosen; pass ``indices`` to supply them.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib as L


def _pose_dtype(t):
    if t.dtype == torch.float32:
        return L.NC_POSE_F32
    if t.dtype == torch.float64:
        return L.NC_POSE_F64
    raise L.NiceCoreError("c2w must be float32 or float64")


def _strides(a, t, name, n):
    st = t.stride()
    arr = getattr(a, name)
    for k in range(n):
        arr[k] = st[k]


class SampleRaysFn(torch.autograd.Function):
    """(spec, c2w [F,3|4,4], indices [F,n] int64 | None, pix_i, pix_j, depth [K,H,W] | None,
    color [K,H,W,3] | None, frame_ids [F] | None) -> (rays_o, rays_d, gt_depth, gt_color, inside).
    Differentiable w.r.t. c2w only (the images and pixels are data)."""

    @staticmethod
    def forward(ctx, spec, c2w, indices, pix_i, pix_j, depth, color, frame_ids):
        lib = L.load()
        device = c2w.device
        if device.type != "cuda":
            raise L.NiceCoreError("nicecore samples rays on a HIP device; c2w is on " + str(device))
        ctx.set_materialize_grads(False)
        c2w_d = c2w.detach()
        F = c2w_d.shape[0]
        n = spec["n"]
        a = L.NcSampleArgs()
        a.abi_version = L.NC_ABI_VERSION
        a.pose_dtype = _pose_dtype(c2w_d)
        a.n_frames, a.n_per_frame = F, n
        a.H0, a.H1, a.W0, a.W1 = spec["region"]
        a.fx, a.fy, a.cx, a.cy = spec["intrinsics"]
        ctx.cam = spec.get("cam", False)
        if ctx.cam:  # [F, 7] camera tensors (ABI v11): get_camera_from_tensor inside the kernels
            a.cam = c2w_d.data_ptr()
            _strides(a, c2w_d, "cam_stride", 2)
        else:
            a.c2w = c2w_d.data_ptr()
            _strides(a, c2w_d, "c2w_stride", 3)
        keep = [c2w_d]
        if indices is not None:
            indices = indices.to(device=device, dtype=torch.int64).contiguous()
            a.indices = indices.data_ptr()
            keep.append(indices)
        else:
            pix_i = pix_i.to(device=device, dtype=torch.float32).contiguous()
            pix_j = pix_j.to(device=device, dtype=torch.float32).contiguous()
            a.pix_i, a.pix_j = pix_i.data_ptr(), pix_j.data_ptr()
            keep += [pix_i, pix_j]
        if frame_ids is not None:
            frame_ids = frame_ids.to(device=device, dtype=torch.int64).contiguous()
            a.frame_ids = frame_ids.data_ptr()
            keep.append(frame_ids)
        rays_o = torch.empty(F * n, 3, device=device, dtype=c2w_d.dtype)
        rays_d = torch.empty(F * n, 3, device=device, dtype=c2w_d.dtype)
        a.rays_o, a.rays_d = rays_o.data_ptr(), rays_d.data_ptr()
        gt_depth = gt_color = inside = None
        if depth is not None:
            if depth.dtype != torch.float32 or depth.dim() != 3 or depth.device != device:
                raise L.NiceCoreError("depth images must be float32 [K,H,W] on the HIP device")
            a.depth = depth.data_ptr()
            _strides(a, depth, "depth_stride", 3)
            gt_depth = torch.empty(F * n, device=device, dtype=torch.float32)
            a.gt_depth = gt_depth.data_ptr()
        if color is not None:
            if color.dtype != torch.float32 or color.dim() != 4 or color.device != device:
                raise L.NiceCoreError("colour images must be float32 [K,H,W,3] on the HIP device")
            a.color = color.data_ptr()
            _strides(a, color, "color_stride", 4)
            gt_color = torch.empty(F * n, 3, device=device, dtype=torch.float32)
            a.gt_color = gt_color.data_ptr()
        bound = spec.get("bound")
        if bound is not None:
            if depth is None:
                raise L.NiceCoreError("the bbox pre-filter compares against gt depth; pass depth")
            b = torch.as_tensor(bound, dtype=torch.float64).reshape(3, 2).to(device).contiguous()
            keep.append(b)
            a.bound = b.data_ptr()
            inside = torch.empty(F * n, device=device, dtype=torch.bool)
            a.inside = inside.data_ptr()
        stream = L.raw_stream(device)
        L.check(lib.nc_sample_rays_forward(ctypes.byref(a), stream), "nc_sample_rays_forward")
        ctx.args, ctx.keep = a, keep
        ctx.c2w_shape = c2w_d.shape
        ctx.mark_non_differentiable(*[t for t in (gt_depth, gt_color, inside) if t is not None])
        return rays_o, rays_d, gt_depth, gt_color, inside

    @staticmethod
    def backward(ctx, g_o, g_d, *_):
        if not ctx.needs_input_grad[1] or (g_o is None and g_d is None):
            return (None,) * 8
        lib = L.load()
        a = ctx.args
        c2w = ctx.keep[0]
        go = g_o.detach().to(c2w.dtype).contiguous() if g_o is not None else None
        gd = g_d.detach().to(c2w.dtype).contiguous() if g_d is not None else None
        a.g_rays_o = go.data_ptr() if go is not None else None
        a.g_rays_d = gd.data_ptr() if gd is not None else None
        stream = L.raw_stream(c2w.device)
        if ctx.cam:  # d cam written by the pose-gradient launch itself
            gcam = torch.empty(c2w.shape[0], 7, device=c2w.device, dtype=c2w.dtype)
            a.g_cam, a.g_c2w = gcam.data_ptr(), None
            L.check(lib.nc_sample_rays_backward(ctypes.byref(a), stream), "nc_sample_rays_backward")
            return None, gcam, None, None, None, None, None, None
        g34 = torch.empty(c2w.shape[0], 3, 4, device=c2w.device, dtype=c2w.dtype)
        a.g_c2w = g34.data_ptr()
        L.check(lib.nc_sample_rays_backward(ctypes.byref(a), stream), "nc_sample_rays_backward")
        if ctx.c2w_shape[1] == 3:
            g = g34
        else:
            g = torch.zeros(ctx.c2w_shape, device=c2w.device, dtype=c2w.dtype)
            g[:, :3, :] = g34
        return None, g, None, None, None, None, None, None


def _as_frames(c2w):
    """[3|4,4] -> [1,3|4,4]; numpy -> tensor."""
    if not isinstance(c2w, torch.Tensor):
        c2w = torch.as_tensor(c2w)
    return (c2w.unsqueeze(0), True) if c2w.dim() == 2 else (c2w, False)


def sample_frames(H0, H1, W0, W1, n, fx, fy, cx, cy, c2w, depth=None, color=None, frame_ids=None,
                  bound=None, indices=None, device=None):
    """All frames' training rays in one launch.  ``c2w`` [F,3|4,4] (float32 / float64,
    may require grad), ``depth`` [K,H,W] / ``color`` [K,H,W,3] float32 image stacks on
    the device, ``frame_ids`` [F] image slot per pose (default: slot f).  Returns
    (rays_o [F*n,3], rays_d [F*n,3] in c2w's dtype, gt_depth [F*n], gt_color [F*n,3],
    inside [F*n] bool — the Tracker/Mapper bbox pre-filter against ``bound``)."""
    c2w, _ = _as_frames(c2w)
    device = c2w.device if device is None else torch.device(device)
    c2w = c2w.to(device)
    F = c2w.shape[0]
    if indices is None:
        region = (H1 - H0) * (W1 - W0)
        indices = torch.stack([torch.randint(region, (n,), device=device) for _ in range(F)]) if F else \
            torch.empty(0, n, dtype=torch.int64, device=device)
    spec = {"n": n, "region": (H0, H1, W0, W1), "intrinsics": (fx, fy, cx, cy), "bound": bound}
    return SampleRaysFn.apply(spec, c2w, indices, None, None, depth, color, frame_ids)


def sample_frames_from_tensor(H0, H1, W0, W1, n, fx, fy, cx, cy, camera_tensor, depth=None, color=None,
                              frame_ids=None, bound=None, indices=None, device=None):
    """sample_frames for the Tracker's camera tensor(s) [F, 7] or [7] ([qr, qi, qj, qk, tx, ty,
    tz]): get_camera_from_tensor (common.py:163-176) is evaluated inside the sampling kernel
    and its backward inside the pose-gradient kernel (ABI v11), so a tracking iteration's
    camera -> rays -> render -> loss -> d camera chain is library launches only (no torch
    quaternion ops and their autograd nodes).  Same returns as sample_frames; the rays
    backpropagate into ``camera_tensor``."""
    cam = camera_tensor if isinstance(camera_tensor, torch.Tensor) else torch.as_tensor(camera_tensor)
    if cam.dim() == 1:
        cam = cam.unsqueeze(0)
    if cam.dim() != 2 or cam.shape[1] != 7:
        raise L.NiceCoreError("camera tensors must be [7] or [F, 7]")
    device = cam.device if device is None else torch.device(device)
    cam = cam.to(device)
    F = cam.shape[0]
    if indices is None:
        region = (H1 - H0) * (W1 - W0)
        indices = torch.stack([torch.randint(region, (n,), device=device) for _ in range(F)]) if F else \
            torch.empty(0, n, dtype=torch.int64, device=device)
    spec = {"n": n, "region": (H0, H1, W0, W1), "intrinsics": (fx, fy, cx, cy), "bound": bound, "cam": True}
    return SampleRaysFn.apply(spec, cam, indices, None, None, depth, color, frame_ids)


def get_samples(H0, H1, W0, W1, n, H, W, fx, fy, cx, cy, c2w, depth, color, device, indices=None):
    """src/common.py:126-137: n rays of the region H0..H1 x W0..W1 of one frame.
    Returns (rays_o, rays_d, sample_depth, sample_color)."""
    c2w, _ = _as_frames(c2w)
    c2w = c2w.to(device)
    if indices is not None:
        indices = indices.reshape(1, -1)
    d = depth.to(device).reshape(1, H, W) if depth is not None else None
    c = color.to(device).reshape(1, H, W, 3) if color is not None else None
    ro, rd, gd, gc, _ = sample_frames(H0, H1, W0, W1, n, fx, fy, cx, cy, c2w, d, c, indices=indices,
                                      device=device)
    return ro, rd, gd, gc


def get_rays_from_uv(i, j, c2w, H, W, fx, fy, cx, cy, device):
    """src/common.py:74-89: rays through caller pixel coordinates i (column), j (row)."""
    c2w, _ = _as_frames(c2w)
    c2w = c2w.to(device)
    i = i.reshape(1, -1)
    j = j.reshape(1, -1)
    spec = {"n": i.shape[1], "region": (0, 1, 0, 1), "intrinsics": (fx, fy, cx, cy), "bound": None}
    ro, rd, _, _, _ = SampleRaysFn.apply(spec, c2w, None, i, j, None, None, None)
    return ro, rd


def bbox_filter(rays_o, rays_d, gt_depth, gt_color, inside):
    """Tracker.py:108-111 / Mapper.py:588-591: keep the rays whose pre-filter mask is set
    (boolean compaction, as the reference; synchronises on the count)."""
    return rays_o[inside], rays_d[inside], gt_depth[inside], gt_color[inside]
