"""ORACLE — TEST INFRASTRUCTURE ONLY.  Never imported by the product path.

CPU restatement of the reference's training-ray sampling (the inputs of
render_batch_ray), with the pixel draw supplied as indices:

  get_rays_from_uv   src/common.py:74-89
  select_uv          src/common.py:92-108   (torch.randint draw replaced by `indices`)
  get_sample_uv      src/common.py:111-123
  get_samples        src/common.py:126-137
  bbox_inside_mask   src/Tracker.py:100-107 / src/Mapper.py:580-587 (pre-filter)
  frames             the Mapper's per-keyframe loop (Mapper.py:543-577) + torch.cat

Parity status: get_samples / get_rays_from_uv (outputs and the c2w gradient) PINNED
against tests/golden/sampling_*.npz, produced by importing the reference's
src.common in the build container (tests/golden/make_golden_sampling.py).
bbox_inside_mask restates three lines inlined in Tracker/Mapper (not importable
here: colorama / cv2 missing) — its inputs are pinned, the mask expression itself is
a restatement.
"""
from __future__ import annotations

import torch


def get_rays_from_uv(i, j, c2w, fx, fy, cx, cy):
    """common.py:74-89 (float32 dirs; rays in c2w's dtype)."""
    dirs = torch.stack([(i - cx) / fx, -(j - cy) / fy, -torch.ones_like(i)], -1)
    dirs = dirs.reshape(-1, 1, 3)
    rays_d = torch.sum(dirs * c2w[:3, :3], -1)
    rays_o = c2w[:3, -1].expand(rays_d.shape)
    return rays_o, rays_d


def get_samples(H0, H1, W0, W1, indices, fx, fy, cx, cy, c2w, depth, color):
    """common.py:111-137 with select_uv's random draw given as ``indices``."""
    depth = depth[H0:H1, W0:W1]
    color = color[H0:H1, W0:W1]
    i, j = torch.meshgrid(torch.linspace(W0, W1 - 1, W1 - W0), torch.linspace(H0, H1 - 1, H1 - H0),
                          indexing='ij')
    i, j = i.t().reshape(-1), j.t().reshape(-1)
    i, j = i[indices], j[indices]
    d = depth.reshape(-1)[indices]
    c = color.reshape(-1, 3)[indices]
    ro, rd = get_rays_from_uv(i, j, c2w, fx, fy, cx, cy)
    return ro, rd, d, c


def bbox_inside_mask(bound, rays_o, rays_d, gt_depth):
    """Tracker.py:100-107 / Mapper.py:580-587."""
    o = rays_o.detach().unsqueeze(-1)
    d = rays_d.detach().unsqueeze(-1)
    t = (bound.unsqueeze(0) - o) / d
    t, _ = torch.min(torch.max(t, dim=2)[0], dim=1)
    return t >= gt_depth


def frames(H0, H1, W0, W1, indices, fx, fy, cx, cy, c2ws, depths, colors, bound=None, cast_float=True):
    """Mapper.py:543-591: per-frame get_samples, .float(), concatenation, pre-filter mask."""
    ro_l, rd_l, d_l, c_l = [], [], [], []
    for f in range(len(c2ws)):
        ro, rd, d, c = get_samples(H0, H1, W0, W1, indices[f], fx, fy, cx, cy, c2ws[f], depths[f], colors[f])
        if cast_float:
            ro, rd, d, c = ro.float(), rd.float(), d.float(), c.float()
        ro_l.append(ro); rd_l.append(rd); d_l.append(d); c_l.append(c)
    ro, rd, d, c = torch.cat(ro_l), torch.cat(rd_l), torch.cat(d_l), torch.cat(c_l)
    inside = bbox_inside_mask(bound, ro, rd, d) if bound is not None else None
    return ro, rd, d, c, inside


def quad2rotation(quad):
    """common.py:137-160 for a batch [B, 4] of quaternions (qr, qi, qj, qk): the rotation with
    two_s = 2 / |q|^2 (a quaternion off unit norm, as Adam leaves it, still maps to a
    rotation-like matrix the same way as the reference's).  The reference assigns the
    entries into ``torch.zeros(bs, 3, 3)`` (float32, common.py:150), so R is rounded to
    float32 whatever the quaternion's dtype, and its gradient passes that float32 tensor
    (rounded to float32) on the way back; get_camera_from_tensor's torch.cat then promotes
    R to the translation's dtype (common.py:173)."""
    qr, qi, qj, qk = quad[:, 0], quad[:, 1], quad[:, 2], quad[:, 3]
    two_s = 2.0 / (quad * quad).sum(-1)
    rows = [[1 - two_s * (qj ** 2 + qk ** 2), two_s * (qi * qj - qk * qr), two_s * (qi * qk + qj * qr)],
            [two_s * (qi * qj + qk * qr), 1 - two_s * (qi ** 2 + qk ** 2), two_s * (qj * qk - qi * qr)],
            [two_s * (qi * qk - qj * qr), two_s * (qj * qk + qi * qr), 1 - two_s * (qi ** 2 + qj ** 2)]]
    R = torch.stack([torch.stack(r, -1) for r in rows], -2)
    return R.float()


def camera_from_tensor(inputs):
    """common.py:163-176 get_camera_from_tensor: [B, 7] (or [7]) -> [B, 3, 4] (or [3, 4])."""
    one = inputs.dim() == 1
    x = inputs.unsqueeze(0) if one else inputs
    RT = torch.cat([quad2rotation(x[:, :4]).to(x.dtype), x[:, 4:, None]], 2)
    return RT[0] if one else RT
