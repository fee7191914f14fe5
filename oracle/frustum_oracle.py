"""ORACLE — TEST INFRASTRUCTURE ONLY.  Never imported by the product path.

numpy restatement of the Mapper's frustum feature selection,
``Mapper.get_mask_from_c2w`` (src/Mapper.py:100-187), with the same numpy / torch
operations and dtypes, and of the one OpenCV call it makes:

  cv2_remap_linear   cv2.remap(img, mapx, mapy, interpolation=cv2.INTER_LINEAR) as
                     implemented in opencv-python 4.5.5.64 (environment.yaml:159):
                     imgproc/src/imgwarp.cpp RemapInvoker (float maps -> 5-bit fixed
                     point by cvRound) + remapBilinear (float table weights, 4 taps,
                     BORDER_CONSTANT with value 0).

Parity status: PARITY UNPINNED.  The reference's function cannot run in this
container (cv2 is not installed, src/Mapper.py does not import) and the reference
ships no fixture for it; the restatement follows the reference's source line by line
and OpenCV 4.5.5's published algorithm.  The GPU kernel is held to this oracle
(tests/test_frustum.py).
"""
from __future__ import annotations

import numpy as np
import torch


def cv2_remap_linear(img: np.ndarray, mapx: np.ndarray, mapy: np.ndarray) -> np.ndarray:
    """cv2.remap(img[H,W] float32, mapx, mapy, INTER_LINEAR), BORDER_CONSTANT(0)."""
    H, W = img.shape
    fx = mapx.astype(np.float32) * np.float32(32)
    fy = mapy.astype(np.float32) * np.float32(32)

    def cv_round(v):  # saturate_cast<int>(float): round half even, INT_MIN when out of range
        ok = np.abs(v) < np.float32(2147483520.0)
        r = np.rint(np.where(ok, v, 0)).astype(np.int64)
        return np.where(ok, r, -2147483648)

    X, Y = cv_round(fx), cv_round(fy)
    sx = np.clip(X >> 5, -32768, 32767)
    sy = np.clip(Y >> 5, -32768, 32767)
    tx1 = (X & 31).astype(np.float32) * np.float32(1.0 / 32)
    ty1 = (Y & 31).astype(np.float32) * np.float32(1.0 / 32)
    tx0, ty0 = np.float32(1) - tx1, np.float32(1) - ty1
    w = [ty0 * tx0, ty0 * tx1, ty1 * tx0, ty1 * tx1]

    def tap(xx, yy):
        ok = (xx >= 0) & (xx < W) & (yy >= 0) & (yy < H)
        return np.where(ok, img[np.clip(yy, 0, H - 1), np.clip(xx, 0, W - 1)], np.float32(0))

    v = [tap(sx, sy), tap(sx + 1, sy), tap(sx, sy + 1), tap(sx + 1, sy + 1)]
    out = ((v[0] * w[0] + v[1] * w[1]) + v[2] * w[2]) + v[3] * w[3]
    outside = (sx >= W) | (sx + 1 < 0) | (sy >= H) | (sy + 1 < 0)
    return np.where(outside, np.float32(0), out).astype(np.float32)


def get_mask_from_c2w(c2w, key, val_shape, depth_np, bound, H, W, fx, fy, cx, cy):
    """Mapper.py:100-187; returns the bool mask [X, Y, Z] (numpy)."""
    X, Y, Z = torch.meshgrid(torch.linspace(bound[0][0], bound[0][1], val_shape[2]),
                             torch.linspace(bound[1][0], bound[1][1], val_shape[1]),
                             torch.linspace(bound[2][0], bound[2][1], val_shape[0]), indexing='ij')
    points = torch.stack([X, Y, Z], dim=-1).reshape(-1, 3)
    if key == 'grid_coarse':
        return np.ones(tuple(val_shape)[::-1]).astype(bool)
    points_bak = points.clone()
    c2w = c2w.cpu().numpy()
    w2c = np.linalg.inv(c2w)
    ones = np.ones_like(points[:, 0]).reshape(-1, 1)
    homo_vertices = np.concatenate([points, ones], axis=1).reshape(-1, 4, 1)
    cam_cord_homo = w2c @ homo_vertices
    cam_cord = cam_cord_homo[:, :3]
    K = np.array([[fx, .0, cx], [.0, fy, cy], [.0, .0, 1.0]]).reshape(3, 3)
    cam_cord[:, 0] *= -1
    uv = K @ cam_cord
    z = uv[:, -1:] + 1e-5
    uv = uv[:, :2] / z
    uv = uv.astype(np.float32)
    remap_chunk = int(3e4)
    depths = []
    for i in range(0, uv.shape[0], remap_chunk):
        depths += [cv2_remap_linear(depth_np, uv[i:i + remap_chunk, 0], uv[i:i + remap_chunk, 1]).reshape(-1, 1)]
    depths = np.concatenate(depths, axis=0)
    edge = 0
    mask = (uv[:, 0] < W - edge) * (uv[:, 0] > edge) * (uv[:, 1] < H - edge) * (uv[:, 1] > edge)
    zero_mask = (depths == 0)
    depths[zero_mask] = np.max(depths)
    mask = mask & (0 <= -z[:, :, 0]) & (-z[:, :, 0] <= depths + 0.5)
    mask = mask.reshape(-1)
    ray_o = c2w[:3, 3]
    ray_o = torch.from_numpy(ray_o).unsqueeze(0)
    dist = points_bak - ray_o
    dist = torch.sum(dist * dist, axis=1)
    mask2 = dist < 0.5 * 0.5
    mask2 = mask2.cpu().numpy()
    mask = mask | mask2
    return mask.reshape(val_shape[2], val_shape[1], val_shape[0])


def margins(c2w, val_shape, depth_np, bound, H, W, fx, fy, cx, cy):
    """Per-voxel distance (float64) of the mask's decisions from their thresholds,
    [X, Y, Z]: min over |u|, |u-W|, |v|, |v-H|, |z|, |-z - (d + 0.5)| and the
    sub-pixel rounding points of the remap — used to excuse last-ulp disagreements."""
    X, Y, Z = torch.meshgrid(torch.linspace(bound[0][0], bound[0][1], val_shape[2]),
                             torch.linspace(bound[1][0], bound[1][1], val_shape[1]),
                             torch.linspace(bound[2][0], bound[2][1], val_shape[0]), indexing='ij')
    p = torch.stack([X, Y, Z], dim=-1).reshape(-1, 3).double().numpy()
    c2w = c2w.cpu().double().numpy()
    w2c = np.linalg.inv(c2w)
    cam = (w2c[:3, :3] @ p.T + w2c[:3, 3:4]).T
    cam[:, 0] *= -1
    z = cam[:, 2] + 1e-5
    u = (fx * cam[:, 0] + cx * cam[:, 2]) / z
    v = (fy * cam[:, 1] + cy * cam[:, 2]) / z
    fr = lambda t: np.abs((t * 32) - np.floor(t * 32) - 0.5)  # noqa: E731
    d = cv2_remap_linear(depth_np, u.astype(np.float32), v.astype(np.float32)).astype(np.float64)
    m = np.minimum.reduce([np.abs(u), np.abs(u - W), np.abs(v), np.abs(v - H), np.abs(z),
                           np.abs(-z - (d + 0.5)), fr(u) / 32, fr(v) / 32])
    return m.reshape(val_shape[2], val_shape[1], val_shape[0])
