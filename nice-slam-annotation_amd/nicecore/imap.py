"""iMAP* on the HIP core (ABI v8, include/nicecore.h ``nc_imap_*``).

``ImapRenderFn`` = Renderer.render_batch_ray (src/utils/Renderer.py:95-262) with
                   ``slam.nice == False`` and ``occupancy: False`` (configs/imap.yaml:5):
                   one scene MLP (get_model(nice=False), src/conv_onet/config.py:28-32)
                   and volume-density compositing (src/common.py:232-247).
``ImapEvalFn``   = Renderer.eval_points' ``decoders(pi, c_grid=None)`` (Renderer.py:74)
                   = MLP.forward with c_dim = 0 (decoder.py:190-219).

Both are differentiable w.r.t. the rays / points and every parameter of the MLP;
there is no PyTorch fallback.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib as L


def _refuse_nondeterministic(needs_param_grad: bool) -> None:
    """The iMAP* weight gradients are split-K float-atomic sums (csrc/nc_imap.hip), so
    their rounding differs from run to run.  A caller that asked for deterministic
    results (NC_DETERMINISTIC=1 or torch.use_deterministic_algorithms(True), as the NICE
    path honours them) gets an error instead of silently varying gradients, the way
    PyTorch refuses its own nondeterministic kernels in that mode."""
    from .render_fn import deterministic_requested
    if needs_param_grad and deterministic_requested():
        raise L.NiceCoreError("nicecore: the iMAP* path has no deterministic weight-gradient reduction "
                              "(split-K float atomics); unset NC_DETERMINISTIC / "
                              "torch.use_deterministic_algorithms or freeze the MLP parameters")


def imap_params(module) -> list:
    """The iMAP* MLP's parameters in ``parameters()`` order (embedder._B,
    pts_linears[0..3].weight/bias, output_linear.weight/bias), checked against the
    shapes the kernels are built for."""
    if getattr(module, "c_dim", None) != 0 or len(module.pts_linears) != 4 or list(module.skips) or \
            not module.color:
        raise L.NiceCoreError("nicecore's iMAP* path needs MLP(c_dim=0, n_blocks=4, skips=[], color=True)")
    ps = [module.embedder._B]
    for l in module.pts_linears:
        ps += [l.weight, l.bias]
    ps += [module.output_linear.weight, module.output_linear.bias]
    want = [(3, 93), (256, 93), (256,)] + [(256, 256), (256,)] * 3 + [(4, 256), (4,)]
    for p, s in zip(ps, want):
        if tuple(p.shape) != s:
            raise L.NiceCoreError(f"iMAP* parameter of shape {tuple(p.shape)}, kernels need {s}")
    return ps


def _fill_params(d: L.NcImapParams, params, device):
    for p in params:
        if p.device != device or p.dtype != torch.float32 or not p.is_contiguous():
            raise L.NiceCoreError("iMAP* parameters must be contiguous float32 on the render device")
    d.fourier_B = params[0].data_ptr()
    for l in range(4):
        d.lin_w[l] = params[1 + 2 * l].data_ptr()
        d.lin_b[l] = params[2 + 2 * l].data_ptr()
    d.out_w, d.out_b = params[9].data_ptr(), params[10].data_ptr()


def _param_grads(flat, params, needs):
    out, o = [], 0
    for p, n in zip(params, needs):
        k = p.numel()
        out.append(flat[o:o + k].view_as(p) if (n and flat is not None) else None)
        o += k
    return out


class ImapRenderFn(torch.autograd.Function):
    """Inputs (spec, rays_o, rays_d, gt_depth|None, *params) -> (depth f64, var f64, color f32)."""

    @staticmethod
    def forward(ctx, spec, rays_o, rays_d, gt_depth, *params):
        lib = L.load()
        device = rays_o.device
        if device.type != "cuda":
            raise L.NiceCoreError("nicecore renders on a HIP device; tensors are on " + str(device))
        ctx.set_materialize_grads(False)
        _refuse_nondeterministic(any(ctx.needs_input_grad[4:]))
        rays_o = rays_o.detach().float().contiguous()
        rays_d = rays_d.detach().float().contiguous()
        N = rays_o.shape[0]
        a = L.NcImapRenderArgs()
        a.abi_version = L.NC_ABI_VERSION
        need = ctx.needs_input_grad
        a.flags = L.NC_SAVE_FOR_BACKWARD if any(need[1:3] + need[4:]) else 0
        a.n_rays, a.n_strat = N, spec["n_strat"]
        a.rays_o, a.rays_d = rays_o.data_ptr(), rays_d.data_ptr()
        for k, row in enumerate(spec["bound"]):
            a.bound[k][0], a.bound[k][1] = row
        for k, v in enumerate(torch.linspace(0., 1., steps=spec["n_strat"]).tolist()):
            a.t_strat[k] = v
        gt = None
        if gt_depth is not None:
            gt = gt_depth.detach().reshape(-1).float().contiguous()
            a.gt_depth = gt.data_ptr()
        dmax = spec.get("depth_max")
        if dmax is not None:
            dmax = dmax.detach().reshape(1).float().contiguous()
            a.depth_max = dmax.data_ptr()
        zx = spec.get("z_extra")
        if zx is not None:
            zx = zx.detach().double().contiguous()
            a.z_extra, a.n_extra = zx.data_ptr(), zx.shape[-1]
        for name in ("z_out", "weights_out"):
            t = spec.get(name)
            if t is not None:
                setattr(a, name, t.data_ptr())
        _fill_params(a.dec, params, device)
        depth = torch.empty(N, device=device, dtype=torch.float64)
        var = torch.empty(N, device=device, dtype=torch.float64)
        color = torch.empty(N, 3, device=device, dtype=torch.float32)
        a.depth, a.var, a.color = depth.data_ptr(), var.data_ptr(), color.data_ptr()
        nbytes = lib.nc_imap_render_workspace_bytes(ctypes.byref(a))
        if nbytes == 0:
            L.check(-1, "nc_imap_render_workspace_bytes")
        ws = torch.empty(nbytes, device=device, dtype=torch.uint8)
        stream = L.raw_stream(device)
        L.check(lib.nc_imap_render_forward(ctypes.byref(a), ws.data_ptr(), nbytes, stream), "nc_imap_render_forward")
        a.z_out, a.weights_out = None, None
        ctx.args, ctx.ws, ctx.nbytes = a, ws, nbytes
        ctx.keep = (rays_o, rays_d, gt, dmax, zx, params)
        return depth, var, color

    @staticmethod
    def backward(ctx, g_depth, g_var, g_color):
        lib = L.load()
        a = ctx.args
        need = ctx.needs_input_grad
        rays_o, params = ctx.keep[0], ctx.keep[5]
        device = rays_o.device
        gd = g_depth.detach().double().contiguous() if g_depth is not None else None
        gv = g_var.detach().double().contiguous() if g_var is not None else None
        gc = g_color.detach().float().contiguous() if g_color is not None else None
        a.g_depth, a.g_var, a.g_color = (t.data_ptr() if t is not None else None for t in (gd, gv, gc))
        g_ro = g_rd = None
        if need[1] or need[2]:  # computed together
            g_ro, g_rd = torch.empty_like(rays_o), torch.empty_like(rays_o)
        a.g_rays_o = g_ro.data_ptr() if g_ro is not None else None
        a.g_rays_d = g_rd.data_ptr() if g_rd is not None else None
        needs_p = need[4:]
        flat = None
        if any(needs_p):
            flat = torch.zeros(lib.nc_imap_param_count(), device=device, dtype=torch.float32)
            a.dec.grad = flat.data_ptr()
        if rays_o.shape[0] > 0:
            stream = L.raw_stream(device)
            L.check(lib.nc_imap_render_backward(ctypes.byref(a), ctx.ws.data_ptr(), ctx.nbytes, stream),
                    "nc_imap_render_backward")
        elif g_ro is not None:
            g_ro.zero_(); g_rd.zero_()
        a.dec.grad = None
        return (None, g_ro if need[1] else None, g_rd if need[2] else None, None,
                *_param_grads(flat, params, needs_p))


class ImapEvalFn(torch.autograd.Function):
    """Inputs (p, *params) -> raw [P,4] float32 (no bound mask)."""

    @staticmethod
    def forward(ctx, p, *params):
        lib = L.load()
        device = p.device
        if device.type != "cuda":
            raise L.NiceCoreError("nicecore evaluates on a HIP device; points are on " + str(device))
        _refuse_nondeterministic(any(ctx.needs_input_grad[1:]))
        pts = p.detach().reshape(-1, 3).double().contiguous()
        P = pts.shape[0]
        a = L.NcImapPointsArgs()
        a.abi_version = L.NC_ABI_VERSION
        a.flags = L.NC_SAVE_FOR_BACKWARD if any(ctx.needs_input_grad) else 0
        a.n_points, a.pts = P, pts.data_ptr()
        _fill_params(a.dec, params, device)
        raw = torch.empty(P, 4, device=device, dtype=torch.float32)
        a.raw = raw.data_ptr()
        nbytes = lib.nc_imap_points_workspace_bytes(ctypes.byref(a))
        ws = torch.empty(max(nbytes, 1), device=device, dtype=torch.uint8)
        stream = L.raw_stream(device)
        L.check(lib.nc_imap_points_forward(ctypes.byref(a), ws.data_ptr(), nbytes, stream), "nc_imap_points_forward")
        ctx.args, ctx.ws, ctx.nbytes = a, ws, nbytes
        ctx.keep = (pts, params)
        ctx.p_dtype, ctx.p_shape = p.dtype, p.shape
        return raw

    @staticmethod
    def backward(ctx, g_raw):
        lib = L.load()
        a = ctx.args
        pts, params = ctx.keep
        need = ctx.needs_input_grad
        device = pts.device
        gr = g_raw.detach().float().contiguous()
        a.g_raw = gr.data_ptr()
        g_pts = torch.empty_like(pts) if need[0] else None
        a.g_pts = g_pts.data_ptr() if g_pts is not None else None
        flat = None
        if any(need[1:]):
            flat = torch.zeros(lib.nc_imap_param_count(), device=device, dtype=torch.float32)
            a.dec.grad = flat.data_ptr()
        if a.n_points > 0:
            stream = L.raw_stream(device)
            L.check(lib.nc_imap_points_backward(ctypes.byref(a), ctx.ws.data_ptr(), ctx.nbytes, stream),
                    "nc_imap_points_backward")
        a.dec.grad = None
        gp = g_pts.to(ctx.p_dtype).reshape(ctx.p_shape) if g_pts is not None else None
        return (gp, *_param_grads(flat, params, need[1:]))


def eval_points(module, p):
    """MLP.forward(p, c_grid=None) of the iMAP* MLP: raw [P,4]."""
    return ImapEvalFn.apply(p, *imap_params(module))


def render_rays(module, rays_o, rays_d, bound, gt_depth=None, n_strat=32, n_importance=0, depth_max=None):
    """Renderer.render_batch_ray with nice=False, occupancy=False, N_surface=0, lindisp=False,
    perturb=0 (configs/imap.yaml:106-111); N_importance > 0 runs the forward-only first pass,
    sample_pdf (det=True) and the differentiable second pass (Renderer.py:239-259)."""
    from .ops import sample_pdf
    from .render_fn import _bound_rows
    if n_strat + n_importance > L.NC_MAX_SAMPLES:
        raise L.NiceCoreError("nicecore supports N_samples + N_importance <= 64")
    params = imap_params(module)
    spec = {"n_strat": n_strat, "bound": _bound_rows(bound), "depth_max": depth_max}
    if n_importance > 0:
        N = rays_o.shape[0]
        z = torch.empty(N, n_strat, device=rays_o.device, dtype=torch.float64)
        w = torch.empty(N, n_strat, device=rays_o.device, dtype=torch.float32)
        with torch.no_grad():
            ImapRenderFn.apply(dict(spec, z_out=z, weights_out=w), rays_o.detach(), rays_d.detach(),
                               gt_depth.detach() if gt_depth is not None else None,
                               *[p.detach() for p in params])
            z_mid = .5 * (z[..., 1:] + z[..., :-1])
            spec["z_extra"] = sample_pdf(z_mid, w[..., 1:-1], n_importance, det=True)
    return ImapRenderFn.apply(spec, rays_o, rays_d, gt_depth, *params)
