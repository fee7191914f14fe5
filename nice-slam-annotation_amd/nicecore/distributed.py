"""Ray-sharded data parallelism for render_batch_ray (one process per GPU, RCCL).

The reference is single-GPU; the loss of both optimisation loops
is a plain SUM over rays (src/Tracker.py:124-130, src/Mapper.py:605-612), so a
ray batch split across ranks reproduces the single-GPU gradient after a SUM
all-reduce of the gradients -- with one caveat: render_batch_ray uses the
batch-global ``max(gt_depth)`` (Renderer.py:157 far clamp, :194 zero-depth
surface samples).  ``global_depth_max`` all-reduces it (MAX) BEFORE rendering and
the render core takes it through ``depth_max=``.

Exchange per mapper iteration: one MAX of a scalar + one SUM over the grid and
decoder gradients.  Large tensors (grid gradients, 3-23 MB each) are reduced in
place; small ones (decoder parameters) are packed into one flat bucket so the
collective count stays small on xGMI.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_bounds(n: int, rank: int, world: int):
    """Contiguous equal chunks (the first n % world ranks get one extra ray)."""
    base, extra = divmod(n, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def shard(rank: int, world: int, *tensors):
    n = tensors[0].shape[0]
    a, b = shard_bounds(n, rank, world)
    return tuple(t[a:b] for t in tensors)


def global_depth_max(gt_depth: torch.Tensor, group=None, ray_mask=None) -> torch.Tensor:
    """max(gt_depth) over every rank's rays, as a 1-element float32 tensor; with
    ``ray_mask`` over the kept rays only (the compacted batch of the bbox pre-filter)."""
    local = gt_depth.detach().reshape(-1).float()
    if ray_mask is not None:  # no compaction (host sync): dropped rays count as -inf
        local = torch.where(ray_mask.reshape(-1).bool(), local, torch.full_like(local, float("-inf")))
    m = local.max().reshape(1) if local.numel() else torch.full((1,), float("-inf"), device=local.device)
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(m, op=dist.ReduceOp.MAX, group=group)
    return m


def _dense(t):
    dims = sorted((st, sz) for st, sz in zip(t.stride(), t.shape) if sz != 1)
    expect = 1
    for st, sz in dims:
        if st != expect:
            return False
        expect *= sz
    return True


def _shared_bases(grads):
    """Split grads into (flat 1-D ranges to reduce, remaining grads).  The render core
    puts every gradient of one backward call into one buffer (render_fn._GradBuffer:
    grid gradients first, then the decoder parameters), each gradient a dense view of
    a contiguous range of it; gradients whose ranges tile a stretch of the buffer
    without gaps are reduced as that one 1-D range (a single collective, and no
    channels-last views handed to the backend).

    Grouped by STORAGE, not by ``._base``: AccumulateGrad stores a detached alias of
    the gradient it steals, which keeps the storage but not the view's base.  A
    contiguous gradient that is its whole storage (an ordinary one) stays apart."""
    by_store = {}
    rest = []
    for g in grads:
        st = g.untyped_storage()
        whole = g.storage_offset() == 0 and g.numel() * g.element_size() == st.nbytes()
        if (whole and g.is_contiguous()) or not _dense(g):
            rest.append(g)
            continue
        off = g.storage_offset()
        by_store.setdefault((st.data_ptr(), g.dtype, g.device), (g, []))[1].append((off, off + g.numel()))
    ranges = []
    for g0, spans in by_store.values():
        st = g0.untyped_storage()
        flat = torch.empty(0, dtype=g0.dtype, device=g0.device).set_(st, 0, (st.nbytes() // g0.element_size(),))
        spans.sort()
        lo, hi = spans[0]
        for s0, s1 in spans[1:]:
            if s0 == hi:
                hi = s1
            else:
                ranges.append(flat[lo:hi])
                lo, hi = s0, s1
        ranges.append(flat[lo:hi])
    return ranges, rest


def allreduce_grads(tensors, group=None, bucket_bytes: int = 4 << 20):
    """SUM all-reduce of the ``.grad`` of every tensor that has one.

    Buffers fully covered by the gradients (the render core's single gradient
    buffer per backward call) are reduced with one collective each.  Remaining
    gradients larger than ``bucket_bytes`` are reduced in place (async); the small
    ones are packed into flat buckets, reduced, and unpacked."""
    allreduce_grads_async(tensors, group, bucket_bytes)()


def allreduce_grads_async(tensors, group=None, bucket_bytes: int = 4 << 20):
    """``allreduce_grads`` with every collective issued asynchronously; returns the
    function that waits for them (and unpacks the small-gradient buckets).  Work
    enqueued on the current stream between the two overlaps the exchange (bench.py
    N > 1: the decoder weight gradients run while the grid gradients are reduced)."""
    if not (dist.is_initialized() and dist.get_world_size(group) > 1):
        return lambda: None
    grads = [t.grad for t in tensors if t.grad is not None]
    whole, grads = _shared_bases(grads)
    handles = [dist.all_reduce(b, group=group, async_op=True) for b in whole]
    big = [g for g in grads if g.numel() * g.element_size() >= bucket_bytes]
    small = [g for g in grads if g.numel() * g.element_size() < bucket_bytes]
    handles += [dist.all_reduce(g, group=group, async_op=True) for g in big]
    by_dtype = {}
    for g in small:
        by_dtype.setdefault((g.dtype, g.device), []).append(g)
    buckets = []
    for _, gs in by_dtype.items():
        flat = torch.cat([g.reshape(-1) for g in gs])
        handles.append(dist.all_reduce(flat, group=group, async_op=True))
        buckets.append((flat, gs))

    def finish():
        for h in handles:
            h.wait()
        for flat, gs in buckets:
            o = 0
            for g in gs:
                n = g.numel()
                g.copy_(flat[o:o + n].view_as(g))
                o += n
    return finish


def allreduce_rows_async(pairs, group=None):
    """SUM all-reduce of selected voxel rows of channels-last grid gradients, the
    Mapper's frustum feature selection (src/Mapper.py:371-414, configs/nice_slam.yaml
    ``frustum_feature_selection: True``): only the voxels inside the current frame's
    frustum are optimisation variables (``val[mask] = val_grad``), so only their rows are
    exchanged -- SURVEY.md §8e's compacted all-reduce.  ``pairs``: (grad [1, C, D, H, W]
    in channels_last_3d, int64 voxel indices in the grid's z-y-x order).  Rows are
    gathered into one flat buffer (one collective), reduced asynchronously, and written
    back by the returned ``finish()``; other rows keep the rank-local values."""
    if not (dist.is_initialized() and dist.get_world_size(group) > 1):
        return lambda: None
    views = []
    for g, idx in pairs:
        v = g.permute(0, 2, 3, 4, 1)
        if not v.is_contiguous():
            raise ValueError("allreduce_rows_async needs channels_last_3d gradients")
        views.append((v.reshape(-1, g.shape[1]), idx))
    if not views:
        return lambda: None
    C = views[0][0].shape[1]
    n = sum(int(idx.numel()) for _, idx in views)
    flat = torch.empty(n, C, dtype=views[0][0].dtype, device=views[0][0].device)
    o = 0
    for v, idx in views:
        torch.index_select(v, 0, idx, out=flat[o:o + idx.numel()])
        o += idx.numel()
    h = dist.all_reduce(flat, group=group, async_op=True)

    def finish():
        h.wait()
        o = 0
        for v, idx in views:
            v.index_copy_(0, idx, flat[o:o + idx.numel()])
            o += idx.numel()
    return finish
