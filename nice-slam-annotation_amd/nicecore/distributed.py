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


def global_depth_max(gt_depth: torch.Tensor, group=None) -> torch.Tensor:
    """max(gt_depth) over every rank's rays, as a 1-element float32 tensor."""
    local = gt_depth.detach().reshape(-1).float()
    m = local.max().reshape(1) if local.numel() else torch.full((1,), float("-inf"), device=local.device)
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(m, op=dist.ReduceOp.MAX, group=group)
    return m


def _shared_bases(grads):
    """Split grads into (buffers reduced whole, remaining grads): a base tensor whose
    elements are exactly covered by views in ``grads`` (the render core puts every
    gradient of one backward call into one buffer: render_fn._alloc_grads) is
    reduced once instead of per view."""
    by_base = {}
    for g in grads:
        b = g._base
        if b is not None and b.is_contiguous():
            by_base.setdefault(id(b), (b, []))[1].append(g)
    whole, covered = [], set()
    for b, views in by_base.values():
        if sum(v.numel() for v in views) == b.numel() and all(v.dtype == b.dtype for v in views):
            whole.append(b)
            covered.update(id(v) for v in views)
    return whole, [g for g in grads if id(g) not in covered]


def allreduce_grads(tensors, group=None, bucket_bytes: int = 4 << 20):
    """SUM all-reduce of the ``.grad`` of every tensor that has one.

    Buffers fully covered by the gradients (the render core's single gradient
    buffer per backward call) are reduced with one collective each.  Remaining
    gradients larger than ``bucket_bytes`` are reduced in place (async); the small
    ones are packed into flat buckets, reduced, and unpacked."""
    if not (dist.is_initialized() and dist.get_world_size(group) > 1):
        return
    grads = [t.grad for t in tensors if t.grad is not None]
    whole, grads = _shared_bases(grads)
    handles = [dist.all_reduce(b, group=group, async_op=True) for b in whole]
    big = [g for g in grads if g.numel() * g.element_size() >= bucket_bytes]
    small = [g for g in grads if g.numel() * g.element_size() < bucket_bytes]
    handles += [dist.all_reduce(g, group=group, async_op=True) for g in big]
    by_dtype = {}
    for g in small:
        by_dtype.setdefault((g.dtype, g.device), []).append(g)
    for _, gs in by_dtype.items():
        flat = torch.cat([g.reshape(-1) for g in gs])
        dist.all_reduce(flat, group=group)
        o = 0
        for g in gs:
            n = g.numel()
            g.copy_(flat[o:o + n].view_as(g))
            o += n
    for h in handles:
        h.wait()
