"""Touched-voxel (sparse) gradients of feature grids too large for a dense gradient.

The reference's grid gradient is dense -- autograd's grid.grad, or the gradient of the
frustum-selected leaf ``val[mask]`` the Mapper steps Adam on (src/Mapper.py:392-404,
:620-627).  For BASELINE configs[4] (fine / colour grids of ~200M voxels, 26 GB each)
a dense gradient is a 26 GB zero fill per iteration and, over 8 ranks, a 26 GB
all-reduce, while a batch of N rays x 48 samples touches at most 8 corners per lookup.

``SparseGridGrads`` keeps, per grid, a voxel -> row map (int32, D*H*W entries) and a
compact ``[capacity, 32]`` float32 gradient, and hands them to the core through
``nc_grid.grad_rows`` (include/nicecore.h, ABI v5):

* the forward claims one row per touched voxel (``k_grid_gather``) and zero-fills it,
* the backward accumulates the trilinear gradient into the rows (``k_mlp_dx``),
* ``allreduce`` merges the ranks' touched sets into one ascending union on every rank
  (``nc_sparse_rows_merge``: radix sort + scan on the device) and sums the rows with
  one RCCL all-reduce of ``count x 128 B`` per grid,
* ``zero_grad`` resets the map (``nc_sparse_rows_clear``), like ``optimizer.zero_grad``.

Row values equal the dense gradient's entries at ``indices`` (``to_dense`` rebuilds it;
tests/test_gpu_sparse.py checks that against the dense path); the voxel index is
``(z * H + y) * W + x`` of the grid's ``[D, H, W]``, i.e. the row index of the
channels-last view ``grid.permute(0, 2, 3, 4, 1).reshape(-1, 32)`` -- which makes
``coo()`` directly usable with ``torch.optim.SparseAdam`` on that view.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib as L

DEFAULT_KEYS = ("grid_middle", "grid_fine", "grid_color")


class _Rows:
    def __init__(self, grid: torch.Tensor, capacity: int):
        D, H, W = grid.shape[2:]
        self.shape = (int(D), int(H), int(W))
        self.n_voxels = int(D) * int(H) * int(W)
        if self.n_voxels >= 2 ** 31:
            raise L.NiceCoreError("sparse gradient rows support grids of < 2^31 voxels")
        dev = grid.device
        self.device = dev
        self.map = torch.full((self.n_voxels,), -1, dtype=torch.int32, device=dev)
        self.count = torch.zeros(1, dtype=torch.int32, device=dev)
        self.capacity = 0
        self.values = self.row_voxel = None
        self._alloc(capacity)
        self.claim_bound = 0  # upper bound of claimed rows since the last clear

    def _alloc(self, cap: int):
        cap = max(1, min(int(cap), self.n_voxels))
        values = torch.empty(cap, 32, dtype=torch.float32, device=self.device)
        rv = torch.empty(cap, dtype=torch.int64, device=self.device)
        if self.values is not None and self.claim_bound > 0:  # keep claimed rows (row ids stay valid)
            n = min(self.capacity, cap)
            values[:n].copy_(self.values[:n])
            rv[:n].copy_(self.row_voxel[:n])
        self.values, self.row_voxel, self.capacity = values, rv, cap

    def reserve(self, extra_claims: int):
        """Make room for up to ``extra_claims`` more claims before the next clear."""
        need = min(self.claim_bound + int(extra_claims), self.n_voxels)
        if need > self.capacity:
            self._alloc(max(need, min(2 * self.capacity, self.n_voxels)))
        self.claim_bound = need

    def struct(self, values=None, row_voxel=None, count=None, capacity=None) -> L.NcSparseRows:
        r = L.NcSparseRows()
        r.grad_rows = self.map.data_ptr()
        r.n_voxels = self.n_voxels
        r.row_voxel = (row_voxel if row_voxel is not None else self.row_voxel).data_ptr()
        r.row_count = (count if count is not None else self.count).data_ptr()
        r.capacity = capacity if capacity is not None else self.capacity
        r.values = (values if values is not None else self.values).data_ptr()
        return r

    def bind(self, ng: L.NcGrid):
        ng.grad = self.values.data_ptr()
        ng.grad_rows = self.map.data_ptr()
        ng.row_voxel = self.row_voxel.data_ptr()
        ng.row_count = self.count.data_ptr()
        ng.row_capacity = self.capacity
        for a in range(4):
            ng.grad_stride[a] = 0
        ng.grad_stride[0] = 1


class SparseGridGrads:
    """Sparse gradient rows of ``grids[key]`` for ``key in keys`` (default: middle, fine,
    colour).  Pass it as ``sparse_grads=`` to ``Renderer.render_batch_ray`` /
    ``render_batch_loss`` / ``ops.render_rays*`` / ``ops.eval_points``: those grids then
    get no dense ``.grad`` (autograd receives None for them; keep ``requires_grad`` on
    so the graph is recorded) and their gradient accumulates here instead."""

    def __init__(self, grids: dict, keys=DEFAULT_KEYS, capacity: int = 1 << 16):
        self.rows = {}
        for k in keys:
            g = grids.get(k)
            if g is None:
                continue
            if g.dim() != 5 or g.shape[0] != 1 or g.shape[1] != 32 or g.device.type != "cuda":
                raise L.NiceCoreError(f"{k}: sparse gradient rows need a [1,32,D,H,W] grid on a HIP device")
            self.rows[k] = _Rows(g, capacity)
        self.grid_index = {L.GRID_KEYS.index(k): k for k in self.rows}

    # --- core binding (render_fn) -------------------------------------------------
    def covers(self, grid_idx: int) -> bool:
        return grid_idx in self.grid_index

    def bind_forward(self, ng: L.NcGrid, grid_idx: int, n_points: int):
        r = self.rows[self.grid_index[grid_idx]]
        r.reserve(8 * n_points)
        r.bind(ng)

    def bind_backward(self, ng: L.NcGrid, grid_idx: int):
        self.rows[self.grid_index[grid_idx]].bind(ng)

    # --- user API -------------------------------------------------------------------
    def zero_grad(self):
        """Forget every claimed row (nc_sparse_rows_clear: map entries back to -1)."""
        lib = L.load()
        for r in self.rows.values():
            stream = L.raw_stream(r.device)
            st = r.struct()
            L.check(lib.nc_sparse_rows_clear(ctypes.byref(st), stream), "nc_sparse_rows_clear")
            r.claim_bound = 0

    def count(self, key) -> int:
        r = self.rows[key]
        n = int(r.count.item())
        if n > r.capacity:
            raise L.NiceCoreError(f"{key}: {n} touched voxels overflowed {r.capacity} gradient rows")
        return n

    def indices(self, key) -> torch.Tensor:
        """Voxel index (z*H + y)*W + x of each gradient row."""
        return self.rows[key].row_voxel[:self.count(key)]

    def values(self, key) -> torch.Tensor:
        """[count, 32] gradient rows (channel-minor)."""
        return self.rows[key].values[:self.count(key)]

    def coo(self, key) -> torch.Tensor:
        """The gradient as a hybrid sparse COO tensor of shape [D*H*W, 32] (one sparse
        dim, the channels dense): the gradient of the channels-last row view
        grid.permute(0, 2, 3, 4, 1).reshape(-1, 32), e.g. for torch.optim.SparseAdam."""
        r = self.rows[key]
        n = self.count(key)
        return torch.sparse_coo_tensor(r.row_voxel[:n][None], r.values[:n], (r.n_voxels, 32))

    def to_dense(self, key, like: torch.Tensor | None = None) -> torch.Tensor:
        """The dense [1,32,D,H,W] gradient these rows stand for (tests, small grids)."""
        r = self.rows[key]
        D, H, W = r.shape
        flat = torch.zeros(r.n_voxels, 32, dtype=torch.float32, device=r.device)
        n = self.count(key)
        flat.index_add_(0, r.row_voxel[:n], r.values[:n])
        dense = flat.reshape(1, D, H, W, 32).permute(0, 4, 1, 2, 3)
        if like is not None and like.is_contiguous():
            dense = dense.contiguous()
        return dense

    def allreduce(self, group=None):
        """Sum the sparse gradients over the ranks of ``group``: all-gather every rank's
        touched voxels, merge them into one ascending union (identical on all ranks,
        nc_sparse_rows_merge), then one all-reduce of the union's rows per grid.  With
        a backend that cannot reduce device tensors (gloo) the exchange goes through
        host memory."""
        import torch.distributed as dist
        if not dist.is_initialized() or dist.get_world_size(group) == 1:
            return
        self.merge(group)
        host = dist.get_backend(group) == "gloo"
        for key, r in self.rows.items():
            n = self.count(key)  # the union's size (identical on every rank)
            if n:
                v = r.values[:n]
                if host:
                    vh = v.cpu()
                    dist.all_reduce(vh, group=group)
                    v.copy_(vh)
                else:
                    dist.all_reduce(v, group=group)

    def merge(self, group=None):
        """The first half of ``allreduce``: replace every grid's rows by the ascending
        union of all ranks' touched voxels (identical on every rank), with this rank's
        partial gradient rows permuted into it (zero where it has none).  The values
        are not summed (``allreduce`` sums them; ``ShardedSparseGridAdam`` reduce-
        scatters them instead)."""
        import torch.distributed as dist
        if not dist.is_initialized() or dist.get_world_size(group) == 1:
            return
        world = dist.get_world_size(group)
        host = dist.get_backend(group) == "gloo"
        lib = L.load()
        for key, r in self.rows.items():
            stream = L.raw_stream(r.device)
            # every rank contributes a fixed-size block: the largest capacity of any rank
            cap = torch.tensor([r.capacity], dtype=torch.int64, device="cpu" if host else r.device)
            dist.all_reduce(cap, op=dist.ReduceOp.MAX, group=group)
            rank_cap = int(cap.item())
            mine = torch.full((rank_cap,), -1, dtype=torch.int64, device=r.device)
            mine[:r.capacity].copy_(r.row_voxel)
            vox = torch.empty(world * rank_cap, dtype=torch.int64, device=r.device)
            cnt = torch.empty(world, dtype=torch.int32, device=r.device)
            if host:
                vl = [torch.empty(rank_cap, dtype=torch.int64) for _ in range(world)]
                cl = [torch.empty(1, dtype=torch.int32) for _ in range(world)]
                dist.all_gather(vl, mine.cpu(), group=group)
                dist.all_gather(cl, r.count.cpu(), group=group)
                vox.copy_(torch.cat(vl))
                cnt.copy_(torch.cat(cl))
            else:
                dist.all_gather_into_tensor(vox, mine, group=group)
                dist.all_gather_into_tensor(cnt, r.count, group=group)
            out_cap = min(world * rank_cap, r.n_voxels)
            new_vals = torch.empty(out_cap, 32, dtype=torch.float32, device=r.device)
            new_rv = torch.empty(out_cap, dtype=torch.int64, device=r.device)
            new_cnt = torch.zeros(1, dtype=torch.int32, device=r.device)
            nbytes = lib.nc_sparse_merge_temp_bytes(world * rank_cap, r.n_voxels)
            if nbytes == 0:
                L.check(-1, "nc_sparse_merge_temp_bytes")
            temp = torch.empty(nbytes, dtype=torch.uint8, device=r.device)
            sin = r.struct()
            sout = r.struct(values=new_vals, row_voxel=new_rv, count=new_cnt, capacity=out_cap)
            L.check(lib.nc_sparse_rows_merge(ctypes.byref(sin), ctypes.byref(sout), vox.data_ptr(), cnt.data_ptr(),
                                             world, rank_cap, temp.data_ptr(), nbytes, stream),
                    "nc_sparse_rows_merge")
            r.values, r.row_voxel, r.count, r.capacity = new_vals, new_rv, new_cnt, out_cap
            r.claim_bound = out_cap
