"""Host-time breakdown of the drop-in (eager) render step on a GPU box:
the C-ABI calls alone (ctypes round trip + the library's host work + its launches, no
sync) against the Python wrapper around them.

    python tools/host_micro.py [--rays 1000]
"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import torch  # noqa: E402


def per_call(fn, n=400):
    """Host time of one call: each call timed alone with the device idle (synchronised
    before it), so a backed-up launch queue cannot stall the measured enqueue."""
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    tot = 0.0
    for _ in range(n):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        tot += time.perf_counter() - t0
    torch.cuda.synchronize()
    return 1e6 * tot / n


if __name__ == "__main__":
    sys.argv = [sys.argv[0]] + sys.argv[1:]
    args = bench.parse()
    bench.setup_dist(args)
    device = torch.device("cuda", 0)
    from nicecore import _lib as L
    from nicecore import render_fn as RF
    lib = L.load()
    w = bench.build_workload(args, 0, device, 1)
    eager, _ = bench.make_step(w, args, 1, device)
    body = bench.make_step.last_body
    print(f"eager step (pre+body+post): {per_call(eager, 200):8.1f} us enqueue/step")
    # capture the args / workspace of one forward through the Function's ctx
    grids, model, renderer = w["grids"], w["model"], w["renderer"]
    ro, rd, gt, gtc = w["ro"], w["rd"], w["gt"], w["gtc"]
    d, u, c, loss = renderer.render_batch_loss(grids, model, rd, ro, device, args.stage, gt, gtc,
                                               loss="mapper", w_color_loss=0.2, color_term=True)
    node = loss.grad_fn
    a, ws, nb = node.args, node.ws, node.nbytes
    stream = torch.cuda.current_stream(device).cuda_stream
    print(f"nc_render_workspace_bytes:   {per_call(lambda: lib.nc_render_workspace_bytes(ctypes.byref(a))):8.1f} us")
    print(f"nc_render_forward (C + launches): {per_call(lambda: lib.nc_render_forward(ctypes.byref(a), ws.data_ptr(), nb, stream)):8.1f} us")
    tmpl = RF.make_plan(args.stage, model).render_template(device, 32, 16, renderer.bound)
    print(f"NcRenderArgs.from_buffer_copy: {per_call(lambda: L.NcRenderArgs.from_buffer_copy(tmpl)):8.1f} us")
    print(f"make_plan:                   {per_call(lambda: RF.make_plan(args.stage, model)):8.1f} us")
    one = torch.ones((), dtype=torch.float64, device=device)

    def fwd_only():
        with torch.no_grad():
            renderer.render_batch_loss(grids, model, rd, ro, device, args.stage, gt, gtc, loss="mapper",
                                       w_color_loss=0.2, color_term=True)
    print(f"render_batch_loss no_grad:   {per_call(fwd_only):8.1f} us")

    def fwd_grad():
        return renderer.render_batch_loss(grids, model, rd, ro, device, args.stage, gt, gtc, loss="mapper",
                                          w_color_loss=0.2, color_term=True)
    print(f"render_batch_loss (grad):    {per_call(fwd_grad):8.1f} us")
    print(f"body (fwd + backward):       {per_call(body, 200):8.1f} us")
    params = [p for p in model.parameters() if p.requires_grad]
    print(f"params requiring grad: {len(params)}")
