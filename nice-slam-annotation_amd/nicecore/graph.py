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

Streams (the cause of the round-4 ``capture_end`` segfault): torch
records on every leaf's gradient accumulator (its AccumulateGrad node) the stream
that was current when the node was created, and the autograd engine makes that
stream wait on the producer's before it hands the leaf its gradient.  A node lives
as long as any autograd graph that reaches it: a body that keeps its undetached
loss (``out["loss"] = loss``) keeps every call's accumulators alive into the next
call, so accumulators created by eager calls on the default stream are still the
ones the captured backward reaches -- and the engine then makes the legacy default
stream wait on an event of the capturing stream, which a capture does not allow
(HIP crashed in ``hipStreamEndCapture``).  GraphedStep therefore warms up and
captures on ONE stream (accumulators created by the warm-up are on the capture
stream), and refuses, with an error naming the cause, a body whose accumulators
belong to a graph that was alive before the GraphedStep was built.
"""
from __future__ import annotations

import gc
import warnings

import torch

from ._lib import NiceCoreError


def _detach(out):
    """Outputs are kept detached: a live loss would keep the autograd graph of the
    previous iteration (and its AccumulateGrad nodes) alive across replays."""
    if isinstance(out, torch.Tensor):
        return out.detach()
    if isinstance(out, (tuple, list)):
        return type(out)(_detach(o) for o in out)
    return out


_WALK_LIMIT = 200_000  # autograd nodes visited per scan (a bound, not a tuning knob)


def _live_accumulators():
    """AccumulateGrad nodes reachable from every autograd graph alive in the process
    (graphs are held by tensors with a grad_fn; tensors are tracked by the cyclic GC),
    as {node: leaf tensor}."""
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        roots = []
        for o in gc.get_objects():
            try:
                if isinstance(o, torch.Tensor) and o.grad_fn is not None:
                    roots.append(o.grad_fn)
            except Exception:  # objects whose isinstance / attribute access raises
                continue
    seen, acc, stack = set(), {}, roots
    while stack and len(seen) < _WALK_LIMIT:
        n = stack.pop()
        if n is None or n in seen:
            continue
        seen.add(n)
        if type(n).__name__ == "AccumulateGrad":
            acc[n] = n.variable
            continue
        stack.extend(f for f, _ in n.next_functions)
    return acc


class GraphedStep:
    def __init__(self, body, warmup: int = 3, pool=None):
        self.body = body
        self.stream = side = torch.cuda.Stream()
        # accumulators of graphs alive before the warm-up: a pre-hook on each records the
        # stream the engine runs it on (its creation stream) if the body's backward reaches it
        reached = []
        handles = [n.register_prehook(lambda grads, leaf=v: reached.append((leaf, torch.cuda.current_stream())))
                   for n, v in _live_accumulators().items() if v.is_cuda]
        try:
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):  # warm up allocator / autograd outside capture
                for _ in range(max(1, warmup)):
                    _detach(body())
        finally:
            for h in handles:
                h.remove()
        stale = [leaf for leaf, s in reached if s != side]
        if stale:
            shapes = ", ".join(sorted({str(tuple(v.shape)) for v in stale})[:4])
            raise NiceCoreError(
                f"GraphedStep: the body's backward reaches gradient accumulator(s) (leaf shapes {shapes}) of an "
                "autograd graph that was alive before the GraphedStep was built -- typically a loss kept without "
                ".detach() from an earlier eager call (e.g. out['loss'] = loss). Torch runs an accumulator on the "
                "stream it was created on, so the captured backward would wait on that stream (the default stream "
                "cannot join a capture). Keep loss.detach() / loss.item(), or drop the old loss, before building "
                "the GraphedStep.")
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        # the same stream as the warm-up: accumulators the warm-up created (and a body
        # that keeps its own loss carries into the capture) are on the capture stream.
        # thread_local: CUDA calls of other host threads (e.g. a process group's watchdog)
        # during the capture do not invalidate it
        with torch.cuda.graph(self.graph, pool=pool, stream=side, capture_error_mode="thread_local"):
            self.out = _detach(body())

    def __call__(self):
        self.graph.replay()
        return self.out
