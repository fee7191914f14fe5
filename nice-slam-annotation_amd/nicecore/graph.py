"""HIP-graph replay of a render + loss + backward iteration.

The render core never synchronises the host, never allocates device memory
itself and enqueues only on the caller's current stream, so a whole
Tracker / Mapper iteration (``render_batch_ray`` -> loss -> ``backward``) can be
captured once into a hipGraph and replayed: one host launch instead of ~35
kernel launches plus the Python / autograd bookkeeping around them.  This is the
MI355X replacement for what a tracing compiler would do to the reference's
per-iteration Python loop (src/Mapper.py:590-620, src/Tracker.py:100-140).

Usage (inputs live in static tensors that are refilled in place)::

    static_ro.copy_(rays_o); static_rd.copy_(rays_d); static_gt.copy_(gt_depth)
    step = GraphedStep(body)      # body(): zero .grad to None, render, loss, backward
    step()                        # replay; p.grad now holds this iteration's gradients
    optimizer.step()

Constraints of capture (checked by torch): no host synchronisation inside
``body`` (no ``.item()``, no boolean-mask indexing) and fixed shapes.
"""
from __future__ import annotations

import torch


def _detach(out):
    """Outputs are kept detached: a live loss would keep the autograd graph of the
    previous iteration (and its AccumulateGrad nodes) alive across replays."""
    if isinstance(out, torch.Tensor):
        return out.detach()
    if isinstance(out, (tuple, list)):
        return type(out)(_detach(o) for o in out)
    return out


class GraphedStep:
    def __init__(self, body, warmup: int = 3, pool=None):
        self.body = body
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):  # warm up allocator / autograd outside capture
            for _ in range(warmup):
                _detach(body())
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        # thread_local: CUDA calls of other host threads (e.g. a process group's
        # watchdog) during the capture do not invalidate it
        with torch.cuda.graph(self.graph, pool=pool, capture_error_mode="thread_local"):
            self.out = _detach(body())

    def __call__(self):
        self.graph.replay()
        return self.out
