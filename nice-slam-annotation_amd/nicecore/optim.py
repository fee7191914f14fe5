"""The Mapper's optimiser step on the device (nc_adam_step, include/nicecore.h ABI v7).

``Adam`` is a drop-in for the ``torch.optim.Adam`` the Mapper builds over its decoder
parameters and feature grids (src/Mapper.py:462-485: one param group per decoder set /
grid with its own lr, StepLR on top; :625 ``optimizer.step()``).  Its update is the
arithmetic of ``torch.optim.Adam(fused=True)`` (ATen fused_adam_utils.cuh): one
``k_adam_multi`` launch for all parameters (up to 32 per launch) reads param/grad/
moments once and writes param/moments once (28 B per element, HBM-bound), for grids in
either memory format.
State (``step``, ``exp_avg``, ``exp_avg_sq``) and ``state_dict`` follow torch.optim.Adam,
so schedulers and checkpoints keep working.

``SparseGridAdam`` steps the grids whose gradient lives in ``SparseGridGrads`` rows
(C5): ``torch.optim.SparseAdam``'s rule (torch/optim/_functional.py
sparse_adam) on the touched voxels only, with the moments kept in the grid's own
layout.  After ``SparseGridGrads.allreduce`` every rank holds the same union and the
same summed rows, so replicated grids stay identical.

There is no CPU path: the step needs libnicecore.so and a HIP device.  With
``capturable=True`` the step counts live on the device (as torch's capturable Adam) and
``step()`` can be captured in the same hipGraph as render + loss + backward, so a whole
Mapper iteration replays as one graph (the learning rates are then fixed at capture).
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib as L


def _dense_layout(t: torch.Tensor) -> bool:
    """Non-overlapping and dense (any dimension order): a flat [numel] view of its storage."""
    dims = sorted((st, sz) for st, sz in zip(t.stride(), t.shape) if sz != 1)
    expect = 1
    for st, sz in dims:
        if st != expect:
            return False
        expect *= sz
    return True


def _adam_args(mode, lr, beta1, beta2, eps, weight_decay, step) -> L.NcAdamArgs:
    a = L.NcAdamArgs()
    a.abi_version = L.NC_ABI_VERSION
    a.mode = mode
    a.lr, a.beta1, a.beta2 = float(lr), float(beta1), float(beta2)
    a.eps, a.weight_decay, a.step = float(eps), float(weight_decay), float(step)
    return a


def adam_step_(param, grad, exp_avg, exp_avg_sq, *, lr, beta1, beta2, eps, weight_decay, step):
    """One fused Adam update of ``param`` / ``exp_avg`` / ``exp_avg_sq`` in place
    (torch.optim.Adam(fused=True) arithmetic; ``step`` counted from 1).  All four
    tensors: float32 on one HIP device, same shape and strides, non-overlapping and dense."""
    ts = (param, grad, exp_avg, exp_avg_sq)
    for t in ts:
        if t.dtype != torch.float32 or t.device.type != "cuda":
            raise L.NiceCoreError("nc_adam_step: float32 tensors on a HIP device")
        if t.shape != param.shape or t.stride() != param.stride():
            raise L.NiceCoreError("nc_adam_step: param, grad and moments must share shape and strides")
    if not _dense_layout(param):
        raise L.NiceCoreError("nc_adam_step: param must be non-overlapping and dense")
    a = _adam_args(L.NC_ADAM_DENSE, lr, beta1, beta2, eps, weight_decay, step)
    a.n = param.numel()
    a.param, a.grad, a.exp_avg, a.exp_avg_sq = (t.data_ptr() for t in ts)
    stream = L.raw_stream(param.device)
    L.check(L.load().nc_adam_step(ctypes.byref(a), stream), "nc_adam_step")


class Adam(torch.optim.Optimizer):
    """``torch.optim.Adam`` drop-in (lr, betas, eps, weight_decay; per-group lr as the
    Mapper sets it).  amsgrad, maximize and sparse gradients are not supported (the
    Mapper uses none of them)."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, amsgrad=False,
                 maximize=False, capturable=False):
        if amsgrad or maximize:
            raise NotImplementedError("nicecore.optim.Adam: amsgrad / maximize")
        if not (0.0 <= lr and 0.0 <= eps and 0.0 <= betas[0] < 1.0 and 0.0 <= betas[1] < 1.0):
            raise ValueError(f"invalid Adam hyper-parameters lr={lr} betas={betas} eps={eps}")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=False,
                                      maximize=False, capturable=capturable))

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        segs, keep, betas, device = [], [], None, None
        for group in self.param_groups:
            for p in group["params"]:
                g = p.grad
                if g is None:
                    continue
                if g.is_sparse:
                    raise RuntimeError("nicecore.optim.Adam does not support sparse gradients; "
                                       "use SparseGridAdam with SparseGridGrads")
                if p.dtype != torch.float32 or p.device.type != "cuda" or not _dense_layout(p):
                    raise L.NiceCoreError("nicecore.optim.Adam: float32, non-overlapping and dense parameters "
                                          "on a HIP device")
                if betas is None:
                    betas, eps, device = group["betas"], group["eps"], p.device
                elif group["betas"] != betas or group["eps"] != eps or p.device != device:
                    self._flush(segs, betas, eps, device)  # one launch per (betas, eps, device)
                    segs, keep = [], []
                    betas, eps, device = group["betas"], group["eps"], p.device
                st = self.state[p]
                cap = group.get("capturable", False)
                if not st:
                    st["step"] = torch.zeros((), dtype=torch.float32, device=p.device if cap else "cpu")
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                if g.stride() != p.stride() or g.dtype != torch.float32:  # e.g. a contiguous grad of a channels-last grid
                    g = torch.empty_like(p, memory_format=torch.preserve_format).copy_(g)
                    keep.append(g)
                if cap:  # step count on the device, incremented by the launch: graph-capturable
                    step, step_dev = 0.0, st["step"].data_ptr()
                else:
                    st["step"] += 1
                    step, step_dev = float(st["step"]), None
                segs.append((p.data_ptr(), g.data_ptr(), st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr(),
                             p.numel(), float(group["lr"]), float(group["weight_decay"]), step, step_dev))
        if segs:
            self._flush(segs, betas, eps, device)
        return loss

    @staticmethod
    def _flush(segs, betas, eps, device):
        """All segments in one nc_adam_step_multi call (one launch per 32 parameters)."""
        arr = (L.NcAdamSegment * len(segs))(*[L.NcAdamSegment(*s) for s in segs])
        a = _adam_args(L.NC_ADAM_DENSE, 0.0, betas[0], betas[1], eps, 0.0, 1.0)
        stream = L.raw_stream(device)
        L.check(L.load().nc_adam_step_multi(ctypes.byref(a), arr, len(segs), stream), "nc_adam_step_multi")


class SparseGridAdam:
    """``torch.optim.SparseAdam``'s rule for the grids of a ``SparseGridGrads``: each
    ``step()`` updates, per grid, only the voxels in its gradient rows (nc_adam_step,
    NC_ADAM_SPARSE_ROWS).  Equivalent to torch.optim.SparseAdam over the channels-last
    row view ``grid.permute(0, 2, 3, 4, 1).reshape(-1, 32)`` with ``sparse.coo(key)`` as
    its gradient, without materialising either."""

    def __init__(self, grids: dict, sparse, lr=1e-3, betas=(0.9, 0.999), eps=1e-8):
        self.sparse = sparse
        self.lr, self.betas, self.eps = lr, betas, eps
        self.grids, self.state = {}, {}
        for k in sparse.rows:
            g = grids[k]
            _, _, _, H, W = g.shape
            vs = g.stride(4)
            if g.stride(3) != W * vs or g.stride(2) != H * W * vs or not _dense_layout(g):
                raise L.NiceCoreError(f"{k}: SparseGridAdam needs a dense grid with voxel index (z*H+y)*W+x")
            self.grids[k] = g
            self.state[k] = {"step": 0,
                             "exp_avg": torch.zeros_like(g, memory_format=torch.preserve_format),
                             "exp_avg_sq": torch.zeros_like(g, memory_format=torch.preserve_format)}

    @torch.no_grad()
    def step(self):
        lib = L.load()
        beta1, beta2 = self.betas
        for k, g in self.grids.items():
            r = self.sparse.rows[k]
            st = self.state[k]
            st["step"] += 1
            a = _adam_args(L.NC_ADAM_SPARSE_ROWS, self.lr, beta1, beta2, self.eps, 0.0, st["step"])
            a.param, a.grad = g.data_ptr(), r.values.data_ptr()
            a.exp_avg, a.exp_avg_sq = st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr()
            a.row_voxel, a.row_count, a.row_capacity = r.row_voxel.data_ptr(), r.count.data_ptr(), r.capacity
            a.voxel_stride, a.channel_stride = g.stride(4), g.stride(1)
            stream = L.raw_stream(g.device)
            L.check(lib.nc_adam_step(ctypes.byref(a), stream), "nc_adam_step")


class ShardedSparseGridAdam:
    """ZeRO-style ``SparseGridAdam`` for grids replicated on every rank (SURVEY.md §8e,
    C5 on 8 GPUs).  Rank r owns the voxel slab ``[r*V/world, (r+1)*V/world)`` of each
    grid and keeps the Adam moments for that slab only (1/world of the optimiser
    state).  ``step()`` replaces ``SparseGridGrads.allreduce`` + ``SparseGridAdam.step``:

    1. ``sparse.merge``: the ascending union of the ranks' touched voxels, identical
       on every rank (nc_sparse_rows_merge), this rank's partial rows permuted into it;
    2. reduce-scatter of the union's rows to their owners (the union is sorted, so each
       owner's rows are one contiguous range; ranges padded to the longest);
    3. each owner applies SparseAdam's rule to its rows (nc_adam_step, moments
       addressed inside its slab);
    4. all-gather of the updated parameter rows, written into every replica.

    Results are bit-identical to the unsharded ``allreduce`` + ``SparseGridAdam`` (the
    row sums and the elementwise rule are the same).  Grids must be channels-last
    (``[1, 32, D, H, W]`` with channel stride 1), the layout the core's fast path uses.
    With gloo the exchange goes through host memory."""

    def __init__(self, grids: dict, sparse, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, group=None):
        import torch.distributed as dist
        self.sparse, self.group = sparse, group
        self.lr, self.betas, self.eps = lr, betas, eps
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.grids, self.state = {}, {}
        for k in sparse.rows:
            g = grids[k]
            if g.stride(1) != 1 or g.stride(4) != 32 or not _dense_layout(g):
                raise L.NiceCoreError(f"{k}: ShardedSparseGridAdam needs a channels-last [1,32,D,H,W] grid")
            V = sparse.rows[k].n_voxels
            v0, v1 = self.rank * V // self.world, (self.rank + 1) * V // self.world
            self.grids[k] = g
            self.state[k] = {"step": 0, "slab": (v0, v1),
                             "exp_avg": torch.zeros(v1 - v0, 32, device=g.device),
                             "exp_avg_sq": torch.zeros(v1 - v0, 32, device=g.device)}

    @torch.no_grad()
    def step(self):
        import torch.distributed as dist
        lib = L.load()
        beta1, beta2 = self.betas
        world, rank, group = self.world, self.rank, self.group
        self.sparse.merge(group)
        host = world > 1 and dist.get_backend(group) == "gloo"
        for k, g in self.grids.items():
            r = self.sparse.rows[k]
            st = self.state[k]
            st["step"] += 1
            n = self.sparse.count(k)
            vox, vals = r.row_voxel[:n], r.values[:n]
            V = r.n_voxels
            edges = torch.tensor([i * V // world for i in range(world + 1)], dtype=torch.int64, device=g.device)
            cut = torch.searchsorted(vox, edges).tolist()
            sizes = [cut[i + 1] - cut[i] for i in range(world)]
            maxc = max(max(sizes), 1)
            # 2. reduce-scatter the rows to their slab owners
            if world > 1:
                send = torch.zeros(world, maxc, 32, device=g.device)
                for i in range(world):
                    send[i, :sizes[i]] = vals[cut[i]:cut[i + 1]]
                if host:
                    sh = send.cpu()
                    dist.all_reduce(sh, group=group)
                    mine = sh[rank].to(g.device)
                else:
                    mine = torch.empty(maxc, 32, device=g.device)
                    dist.reduce_scatter_tensor(mine, send.view(world * maxc, 32), group=group)
            else:
                mine = vals
            # 3. SparseAdam rule on the owned rows; moments addressed inside the slab
            own = sizes[rank]
            my_vox = vox[cut[rank]:cut[rank + 1]]
            cnt = torch.tensor([own], dtype=torch.int32, device=g.device)
            v0 = st["slab"][0]
            a = _adam_args(L.NC_ADAM_SPARSE_ROWS, self.lr, beta1, beta2, self.eps, 0.0, st["step"])
            a.param, a.grad = g.data_ptr(), mine.data_ptr()
            a.exp_avg = st["exp_avg"].data_ptr() - v0 * 32 * 4
            a.exp_avg_sq = st["exp_avg_sq"].data_ptr() - v0 * 32 * 4
            a.row_voxel, a.row_count, a.row_capacity = my_vox.data_ptr(), cnt.data_ptr(), own
            a.voxel_stride, a.channel_stride = 32, 1
            stream = L.raw_stream(g.device)
            L.check(lib.nc_adam_step(ctypes.byref(a), stream), "nc_adam_step")
            if world == 1:
                continue
            # 4. all-gather the updated rows into every replica
            rows = g.permute(0, 2, 3, 4, 1).reshape(-1, 32)  # a view (channels-last)
            upd = torch.zeros(maxc, 32, device=g.device)
            upd[:own] = rows[my_vox]
            if host:
                parts = [torch.empty(maxc, 32) for _ in range(world)]
                dist.all_gather(parts, upd.cpu(), group=group)
                allu = torch.stack(parts).to(g.device)
            else:
                allu = torch.empty(world, maxc, 32, device=g.device)
                dist.all_gather_into_tensor(allu.view(world * maxc, 32), upd, group=group)
            for i in range(world):
                if i != rank and sizes[i]:
                    rows[vox[cut[i]:cut[i + 1]]] = allu[i, :sizes[i]]
