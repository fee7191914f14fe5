"""Where the host time of one eager drop-in step goes (bench.py C2 workload): the
NiceRenderFn forward / backward Python bodies, and inside them the library calls
(nc_render_forward / nc_render_backward: argument checks + kernel launches).  The
backward runs on autograd's device thread, so it is timed by wrapping it, not by
cProfile.

    python tools/host_split.py [--steps 200]"""
import os
import sys
import time
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import torch  # noqa: E402

ACC = defaultdict(float)


def timed(name, fn):
    def w(*a, **k):
        t0 = time.perf_counter()
        try:
            return fn(*a, **k)
        finally:
            ACC[name] += time.perf_counter() - t0
    return w


class LibProxy:
    def __init__(self, lib):
        self._lib = lib

    def __getattr__(self, name):
        f = getattr(self._lib, name)
        return timed("lib." + name, f) if name.startswith("nc_render") else f


def main():
    args = bench.parse()
    world, rank, local = bench.setup_dist(args)
    device = torch.device("cuda", 0)
    from nicecore import _lib as L
    from nicecore import render_fn as RF
    lib = L.load()
    proxy = LibProxy(lib)
    L.load = lambda: proxy
    RF.L.load = L.load
    RF.NiceRenderFn.forward = staticmethod(timed("fn.forward", RF.NiceRenderFn.forward))
    RF.NiceRenderFn.backward = staticmethod(timed("fn.backward", RF.NiceRenderFn.backward))
    w = bench.build_workload(args, rank, device, world)
    grids, model, r = w["grids"], w["model"], w["renderer"]
    ro, rd, gt, gtc = w["ro"], w["rd"], w["gt"], w["gtc"]
    leaves = [p for p in model.parameters() if p.requires_grad] + [g for g in grids.values() if g.requires_grad]
    leaves += [ro, rd]

    def zero():
        for t in leaves:
            t.grad = None

    def fused():
        d, u, c, loss = r.render_batch_loss(grids, model, rd, ro, device, "color", gt, gtc, loss="mapper",
                                            w_color_loss=0.2, color_term=True)
        loss.backward()

    def ref():
        depth, unc, color = r.render_batch_ray(grids, model, rd, ro, device, "color", gt)
        m = gt > 0
        loss = torch.abs(gt[m] - depth[m]).sum()
        loss += 0.2 * torch.abs(gtc - color).sum()
        loss.backward()

    parts = {"zero": zero, "fused": fused, "ref": ref}
    for name in ("fused", "ref"):
        for _ in range(20):
            zero()
            parts[name]()
        torch.cuda.synchronize()
        ACC.clear()
        n = args.steps
        tz = tb = 0.0
        t0 = time.perf_counter()
        for _ in range(n):
            a = time.perf_counter()
            zero()
            b = time.perf_counter()
            parts[name]()
            c = time.perf_counter()
            tz += b - a
            tb += c - b
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        print(f"== {name}: wall {1e3 * (t1 - t0) / n:.4f} ms/step; grad=None loop {1e3 * tz / n:.4f}; "
              f"step body {1e3 * tb / n:.4f}")
        for k, v in sorted(ACC.items(), key=lambda kv: -kv[1]):
            print(f"   {k:28s} {1e3 * v / n:.4f} ms/step")


if __name__ == "__main__":
    main()
