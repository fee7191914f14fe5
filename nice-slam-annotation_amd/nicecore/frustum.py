"""Frustum feature selection on the HIP core (ABI v4, nc_frustum_mask).

``FrustumSelector.get_mask_from_c2w(c2w, key, val_shape, depth_np)`` has the signature
and result of ``Mapper.get_mask_from_c2w`` (src/Mapper.py:100-187): a bool mask
[X, Y, Z] of the grid voxels inside the camera frustum (depth-tested against the
frame's depth image) or within 0.5 m of the camera centre.  Here the mask is a device
tensor (a permuted view of the kernel's [Z, Y, X] output, so ``.permute(2, 1, 0)`` as
the Mapper does at :394 gives back the contiguous grid-order mask), and the per-voxel
work -- projection, cv2.remap of the depth image, depth test -- runs as two kernels
instead of numpy + OpenCV over every voxel on the host.

Host-side, exactly as the reference: the voxel coordinate tables (torch.linspace on
the CPU, cached per bound and shape) and w2c = np.linalg.inv(c2w) in float32.

``MaskedGrid`` is the rest of the Mapper's frustum feature selection, the per-iteration
part, on the device (nc_grid_rows): ``select`` = ``val[mask].clone()``
(Mapper.py:393-404), ``scatter_`` = ``val[mask] = val_grad`` with its autograd
(:491-500; backward ``grad[mask]``), ``write_back_`` = the detached write after the
optimiser step (:633-642).  The voxel list is taken from the mask once per frame
(``mask.nonzero()``, one host sync), so no iteration synchronises on a boolean index as
ATen's index_put does; the packed tensor has val[mask]'s layout ([C][n], channel-major),
so optimiser state and checkpoints are interchangeable with the reference's.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib as L


class FrustumSelector:
    def __init__(self, bound, H, W, fx, fy, cx, cy, device="cuda"):
        self.bound = bound
        self.H, self.W, self.fx, self.fy, self.cx, self.cy = H, W, fx, fy, cx, cy
        self.device = torch.device(device)
        self._tables = {}
        self._scratch = None

    def _axis_tables(self, val_shape):
        key = tuple(int(s) for s in val_shape)
        t = self._tables.get(key)
        if t is None:
            b = self.bound
            t = (torch.linspace(b[0][0], b[0][1], key[2]).to(self.device),   # Mapper.py:116-118
                 torch.linspace(b[1][0], b[1][1], key[1]).to(self.device),
                 torch.linspace(b[2][0], b[2][1], key[0]).to(self.device))
            self._tables[key] = t
        return t

    def grid_mask(self, c2w, key, val_shape, depth):
        """The mask in the grid's own [Z, Y, X] order (bool, device)."""
        val_shape = tuple(int(s) for s in val_shape)
        if key == 'grid_coarse':  # Mapper.py:121-123
            return torch.ones(val_shape, dtype=torch.bool, device=self.device)
        lib = L.load()
        if self.device.type != "cuda":
            raise L.NiceCoreError("nicecore selects frustum features on a HIP device")
        xs, ys, zs = self._axis_tables(val_shape)
        c2w_np = c2w.detach().cpu().numpy() if isinstance(c2w, torch.Tensor) else np.asarray(c2w)
        w2c = np.linalg.inv(c2w_np)  # Mapper.py:126, in c2w's dtype
        depth_t = torch.as_tensor(depth).to(self.device, torch.float32)
        if depth_t.dim() != 2:
            raise L.NiceCoreError("depth must be an [H, W] image")
        a = L.NcFrustumArgs()
        a.abi_version = L.NC_ABI_VERSION
        a.nx, a.ny, a.nz = val_shape[2], val_shape[1], val_shape[0]
        a.xs, a.ys, a.zs = xs.data_ptr(), ys.data_ptr(), zs.data_ptr()
        w = w2c.astype(np.float32).reshape(-1)
        for k in range(16):
            a.w2c[k] = float(w[k])
        o = c2w_np[:3, 3].astype(np.float32)
        for k in range(3):
            a.cam_o[k] = float(o[k])
        a.fx, a.fy, a.cx, a.cy = float(self.fx), float(self.fy), float(self.cx), float(self.cy)
        a.depth = depth_t.data_ptr()
        a.H, a.W = depth_t.shape
        a.depth_stride[0], a.depth_stride[1] = depth_t.stride()
        mask = torch.empty(val_shape, dtype=torch.bool, device=self.device)
        if self._scratch is None:
            self._scratch = torch.zeros(1, dtype=torch.int32, device=self.device)
        a.mask = mask.data_ptr()
        a.scratch = self._scratch.data_ptr()
        stream = L.raw_stream(self.device)
        L.check(lib.nc_frustum_mask(ctypes.byref(a), stream), "nc_frustum_mask")
        self._keep = depth_t
        return mask

    def get_mask_from_c2w(self, c2w, key, val_shape, depth_np):
        """Mapper.py:100-187: bool mask [X, Y, Z] (device tensor view)."""
        return self.grid_mask(c2w, key, val_shape, depth_np).permute(2, 1, 0)


def _rows_call(op, grid, rows, packed):
    lib = L.load()
    if grid.device.type != "cuda":
        raise L.NiceCoreError("nicecore moves grid rows on a HIP device")
    if grid.dim() != 5 or grid.shape[0] != 1 or grid.dtype != torch.float32:
        raise L.NiceCoreError(f"grid must be [1,C,D,H,W] float32, got {tuple(grid.shape)} {grid.dtype}")
    a = L.NcGridRowsArgs()
    a.abi_version = L.NC_ABI_VERSION
    a.op = op
    a.n_rows = rows.numel()
    a.rows = rows.data_ptr()
    a.grid = grid.data_ptr()
    a.channels = grid.shape[1]
    for k in range(3):
        a.dims[k] = grid.shape[2 + k]
    for k in range(4):
        a.stride[k] = grid.stride(1 + k)
    a.packed = packed.data_ptr() if packed is not None else None
    L.check(lib.nc_grid_rows(ctypes.byref(a), L.raw_stream(grid.device)), "nc_grid_rows")


class _RowsScatter(torch.autograd.Function):
    """val[mask] = val_grad in place (index_put), differentiable: d val_grad = grad[mask]
    and d val = grad with the masked voxels zeroed -- IndexPutBackward's two outputs."""

    @staticmethod
    def forward(ctx, grid, packed, rows):
        _rows_call(L.NC_ROWS_SCATTER, grid, rows, packed.detach().contiguous())
        ctx.mark_dirty(grid)
        ctx.rows = rows
        ctx.packed_shape = packed.shape
        return grid

    @staticmethod
    def backward(ctx, g):
        d_packed = d_grid = None
        if ctx.needs_input_grad[1]:
            d_packed = torch.empty(ctx.packed_shape, device=g.device, dtype=g.dtype)
            _rows_call(L.NC_ROWS_GATHER, g, ctx.rows, d_packed)
        if ctx.needs_input_grad[0]:
            d_grid = g.clone()
            _rows_call(L.NC_ROWS_ZERO, d_grid, ctx.rows, None)
        return d_grid, d_packed, None


class MaskedGrid:
    """One grid's frustum selection (Mapper.py:393-404): ``mask`` is the grid-order
    [D, H, W] bool mask (FrustumSelector.grid_mask, or ``mask_xyz.permute(2, 1, 0)`` of
    get_mask_from_c2w's result, as Mapper.py:394 permutes it), or the 5-D channel-repeated
    mask the Mapper builds; the voxel list is formed once here."""

    def __init__(self, mask):
        m = mask
        if m.dim() == 5:  # [1, C, D, H, W] channel-repeated: every channel has the same voxels
            m = m[0, 0]
        if m.dim() != 3:
            raise L.NiceCoreError("frustum mask must be [D, H, W] (or [1, C, D, H, W])")
        self.shape = tuple(m.shape)
        self.rows = m.reshape(-1).nonzero().squeeze(1).contiguous()

    @property
    def n(self) -> int:
        return self.rows.numel()

    def _check(self, grid):
        if tuple(grid.shape[2:]) != self.shape:
            raise L.NiceCoreError(f"grid {tuple(grid.shape)} does not match the mask {self.shape}")

    def select(self, grid) -> torch.Tensor:
        """``val[mask].clone()`` (1-D, C * n, channel-major), a fresh leaf tensor."""
        self._check(grid)
        out = torch.empty(grid.shape[1] * self.n, device=grid.device, dtype=grid.dtype)
        _rows_call(L.NC_ROWS_GATHER, grid.detach(), self.rows, out)
        return out

    def scatter_(self, grid, val_grad) -> torch.Tensor:
        """``val[mask] = val_grad`` (in place on ``grid``; autograd records it, so a render
        of ``grid`` back-propagates into ``val_grad``).  Returns ``grid``."""
        self._check(grid)
        if val_grad.numel() != grid.shape[1] * self.n:
            raise L.NiceCoreError("val_grad must hold C x n values (val[mask]'s layout)")
        return _RowsScatter.apply(grid, val_grad, self.rows)

    def write_back_(self, grid, val_grad) -> torch.Tensor:
        """``val = val.detach(); val[mask] = val_grad.clone().detach()``: the updated rows
        into the grid after the optimiser step, outside autograd.  Returns the detached grid."""
        self._check(grid)
        g = grid.detach()
        _rows_call(L.NC_ROWS_SCATTER, g, self.rows, val_grad.detach().contiguous())
        return g

