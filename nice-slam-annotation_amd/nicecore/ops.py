"""Functional entry points of the render core (HIP only, no fallback)."""
from __future__ import annotations

import torch

from . import _lib as L
from .render_fn import NiceEvalFn, NiceRenderFn, make_plan, param_inputs


def _grid_args(c):
    return [c.get(k) if c is not None else None for k in L.GRID_KEYS]


def eval_points(decoders, p, c_grid, stage='middle', deterministic=None, sparse_grads=None):
    """NICE.forward(p, c_grid, stage) (src/conv_onet/models/decoder.py:336-370):
    raw [P,4] float32 for points p ([P,3] or [1,P,3]); differentiable w.r.t. p,
    the grids and the decoder parameters.  ``deterministic``, ``sparse_grads``: see
    render_rays."""
    plan = make_plan(stage, decoders)
    spec = {"plan": plan, "deterministic": deterministic, "sparse": sparse_grads}
    return NiceEvalFn.apply(spec, p, *_grid_args(c_grid), *plan.flat_params())


def _importance_depths(decoders, c, rays_o, rays_d, bound, stage, gt_depth, n_strat, n_surf,
                       depth_max, n_importance, det, lindisp=False, t_rand=None, ray_valid=None):
    """Renderer.py:239-250: a forward-only first pass over the stratified (+ surface)
    samples, then sample_pdf over its weights without the first and last sample at the
    mid-points of its depths.  Returns the N_importance depths [N, n_importance]."""
    N = rays_o.shape[0]
    S = n_strat + n_surf
    dev = rays_o.device
    z = torch.empty(N, S, device=dev, dtype=torch.float64)
    w = torch.empty(N, S, device=dev, dtype=torch.float32)
    plan = make_plan(stage, decoders)
    spec = {"plan": plan, "n_strat": n_strat, "n_surf": n_surf, "bound": bound, "depth_max": depth_max,
            "z_out": z, "weights_out": w, "lindisp": lindisp, "t_rand": t_rand, "ray_valid": ray_valid}
    with torch.no_grad():
        grids = [g.detach() if g is not None else None for g in _grid_args(c)]
        NiceRenderFn.apply(spec, rays_o.detach(), rays_d.detach(),
                           gt_depth.detach() if gt_depth is not None else None, *grids,
                           *[p.detach() for p in plan.flat_params()])
        z_mid = .5 * (z[..., 1:] + z[..., :-1])
        return sample_pdf(z_mid, w[..., 1:-1], n_importance, det=det)


def _t_rand(t_rand, perturb, n_rays, n_strat, device):
    """The stratified samples' jitter draws (Renderer.py:211-219) when perturb > 0: the
    caller's ``t_rand``, or torch.rand([N, N_samples]) on the CPU's default generator moved
    to the device, as the reference draws them.  None when perturb == 0 -- the reference
    does not jitter then, so a ``t_rand`` passed with perturb == 0 is not used."""
    if perturb <= 0.:
        return None
    if t_rand is None:
        t_rand = torch.rand(n_rays, n_strat)
    t_rand = t_rand.detach().to(device=device, dtype=torch.float32).reshape(n_rays, n_strat).contiguous()
    return t_rand


def render_rays(decoders, c, rays_o, rays_d, bound, stage, gt_depth=None, n_strat=32,
                n_surf=16, depth_max=None, deterministic=None, sparse_grads=None, n_importance=0,
                perturb=0., lindisp=False, t_rand=None, param_grads=None, ray_mask=None):
    """Renderer.render_batch_ray core (src/utils/Renderer.py:95-262), occupancy = True.
    Returns (depth float64 [N], uncertainty float64 [N], color float32 [N,3]).

    ``lindisp``: stratified depths linear in disparity (Renderer.py:208-209).  ``perturb``
    > 0 jitters them inside their intervals (Renderer.py:211-219) with ``t_rand``
    ([N, n_strat] uniform draws; default torch.rand on the CPU generator, as the
    reference); with perturb == 0 there is no jitter and ``t_rand`` is not used.

    ``depth_max``: optional device scalar replacing the batch-global max(gt_depth)
    (Renderer.py:157, :194) -- pass the all-reduced max when a batch is sharded.

    ``deterministic``: grid gradients by an ordered per-voxel reduction (bit-identical
    run to run) instead of float atomics; None = the environment variable
    ``NC_DETERMINISTIC=1`` or ``torch.use_deterministic_algorithms(True)``.

    ``sparse_grads``: a ``nicecore.sparse.SparseGridGrads``; the grids it covers get
    their gradient as touched-voxel rows there instead of a dense ``.grad``.

    ``n_importance`` > 0: hierarchical sampling (Renderer.py:239-259) -- a forward-only
    pass, ``sample_pdf`` (deterministic u when ``perturb`` == 0, as the reference), and
    the differentiable render over the sorted union of both sample sets.

    ``param_grads``: "direct" (default) or "autograd" -- how the decoder parameters get
    their ``.grad`` (render_fn.param_inputs).

    ``ray_mask``: optional [N] bool / uint8 device tensor, the callers' bbox pre-filter
    (Tracker.py:100-111, Mapper.py:580-596) applied as a mask instead of ``rays[mask]``:
    rays where it is False are dropped from the batch depth max, the loss and every
    gradient, and report depth / uncertainty / colour 0; the kept rays get what the
    compacted batch would (no host sync: the call stays graph-capturable)."""
    if stage == 'coarse':
        gt_depth = None
    ns = n_surf if gt_depth is not None else 0
    if n_strat + ns + n_importance > L.NC_MAX_SAMPLES or ns > L.NC_MAX_SURF:
        raise L.NiceCoreError("nicecore supports N_samples + N_surface + N_importance <= 64 (N_surface <= 32)")
    plan = make_plan(stage, decoders)
    tr = _t_rand(t_rand, perturb, rays_o.shape[0], n_strat, rays_o.device)
    spec = {"plan": plan, "n_strat": n_strat, "n_surf": ns, "bound": bound, "depth_max": depth_max,
            "deterministic": deterministic, "sparse": sparse_grads, "lindisp": bool(lindisp), "t_rand": tr,
            "ray_valid": ray_mask}
    if n_importance > 0:  # sample_pdf(det=(perturb == 0.)), Renderer.py:247
        spec["z_extra"] = _importance_depths(decoders, c, rays_o, rays_d, bound, stage, gt_depth, n_strat, ns,
                                             depth_max, n_importance, det=(perturb <= 0.),
                                             lindisp=bool(lindisp), t_rand=tr, ray_valid=ray_mask)
    return NiceRenderFn.apply(spec, rays_o, rays_d, gt_depth, *_grid_args(c),
                              *param_inputs(spec, plan, rays_o.device, param_grads))


_LOSS_KINDS = {"mapper": L.NC_LOSS_MAPPER, "tracker": L.NC_LOSS_TRACKER}


def render_rays_loss(decoders, c, rays_o, rays_d, bound, stage, target_depth, loss="mapper",
                     target_color=None, w_color=0.2, color_term=False, handle_dynamic=False,
                     gt_depth="target", n_strat=32, n_surf=16, depth_max=None, deterministic=None,
                     sparse_grads=None, n_importance=0, perturb=0., defer_param_grads=None, lindisp=False,
                     t_rand=None, param_grads=None, ray_mask=None):
    """render_rays + the rendering loss in the same launches.  Returns (depth, uncertainty,
    color, loss) with ``loss`` a float64 device scalar that backpropagates into the
    grids / decoders / rays like the reference's loss expression:

    ``loss="mapper"``  (src/Mapper.py:603-612)
        sum_{target_depth>0} |target_depth - depth|  [+ w_color * sum |target_color - color|]
    ``loss="tracker"`` (src/Tracker.py:117-131; uncertainty detached)
        tmp = |target_depth - depth| / sqrt(uncertainty + 1e-10)
        mask = target_depth > 0 [& tmp < 10 * tmp.median()]  (handle_dynamic)
        sum_mask tmp  [+ w_color * sum_mask |target_color - color|]

    ``color_term`` adds the colour term (Mapper: stage == 'color' or not nice; Tracker:
    use_color_in_tracking).  ``gt_depth`` is the depth that guides the surface samples;
    by default the target itself (the tracker and the non-coarse mapper); the coarse
    mapper renders with None.  ``defer_param_grads``: a render_fn.DeferParamGrads that
    takes the decoder weight gradients out of ``backward()`` (data-parallel overlap).
    ``param_grads``, ``ray_mask``: see render_rays (a dropped ray is in neither loss term
    nor the tracker's median)."""
    if loss not in _LOSS_KINDS:
        raise L.NiceCoreError(f"loss must be one of {sorted(_LOSS_KINDS)}")
    if handle_dynamic and loss != "tracker":
        raise L.NiceCoreError("handle_dynamic is the tracker's outlier mask")
    if color_term and target_color is None:
        raise L.NiceCoreError("color_term needs target_color")
    flags = (L.NC_LOSS_COLOR if color_term else 0) | (L.NC_LOSS_DYNAMIC if handle_dynamic else 0)
    if isinstance(gt_depth, str):
        gt_depth = target_depth
    if stage == 'coarse':
        gt_depth = None
    ns = n_surf if gt_depth is not None else 0
    if n_strat + ns + n_importance > L.NC_MAX_SAMPLES or ns > L.NC_MAX_SURF:
        raise L.NiceCoreError("nicecore supports N_samples + N_surface + N_importance <= 64 (N_surface <= 32)")
    plan = make_plan(stage, decoders)
    tr = _t_rand(t_rand, perturb, rays_o.shape[0], n_strat, rays_o.device)
    spec = {"plan": plan, "n_strat": n_strat, "n_surf": ns, "bound": bound, "depth_max": depth_max,
            "deterministic": deterministic, "sparse": sparse_grads,
            "loss": (_LOSS_KINDS[loss], flags, w_color, target_depth, target_color if color_term else None),
            "defer": defer_param_grads, "lindisp": bool(lindisp), "t_rand": tr, "ray_valid": ray_mask}
    if n_importance > 0:
        spec["z_extra"] = _importance_depths(decoders, c, rays_o, rays_d, bound, stage, gt_depth, n_strat, ns,
                                             depth_max, n_importance, det=(perturb <= 0.),
                                             lindisp=bool(lindisp), t_rand=tr, ray_valid=ray_mask)
    return NiceRenderFn.apply(spec, rays_o, rays_d, gt_depth, *_grid_args(c),
                              *param_inputs(spec, plan, rays_o.device, param_grads))


def sample_pdf(bins, weights, N_samples, det=False, device=None, u=None):
    """Hierarchical sampling (src/common.py:19-63) on the HIP core (``nc_sample_pdf``):
    ``N_samples`` inverse-CDF samples per row of the piecewise-constant pdf
    ``weights + 1e-5`` over ``bins``.  ``bins`` [..., nb] float64 (the reference passes
    the mid-points of its float64 sample depths), ``weights`` [..., nb - 1] float32.
    ``det=False`` draws ``u`` uniformly on the device unless it is given (the reference
    draws it with ``torch.rand`` on the CPU).  Returns float64 [..., N_samples]; no
    gradient (the reference detaches the samples, Renderer.py:247)."""
    import ctypes
    lib = L.load()
    dev = bins.device
    if dev.type != "cuda":
        raise L.NiceCoreError("sample_pdf runs on a HIP device; bins are on " + str(dev))
    lead = bins.shape[:-1]
    nb = bins.shape[-1]
    b = bins.detach().reshape(-1, nb).to(torch.float64).contiguous()
    w = weights.detach().reshape(-1, weights.shape[-1]).to(torch.float32).contiguous()
    if w.shape != (b.shape[0], nb - 1):
        raise L.NiceCoreError(f"weights must be [..., {nb - 1}] for {nb} bins, got {tuple(weights.shape)}")
    n = b.shape[0]
    uu = None
    if not det:
        uu = (torch.rand(n, N_samples, device=dev) if u is None
              else u.detach().reshape(n, N_samples).to(device=dev, dtype=torch.float32).contiguous())
    out = torch.empty(n, N_samples, device=dev, dtype=torch.float64)
    a = L.NcPdfArgs(abi_version=L.NC_ABI_VERSION, det=1 if det else 0, n_rays=n, n_bins=nb,
                    n_samples=N_samples, bins=b.data_ptr(), bins_stride=nb, weights=w.data_ptr(),
                    weights_stride=nb - 1, u=uu.data_ptr() if uu is not None else None,
                    u_stride=N_samples, samples=out.data_ptr(), samples_stride=N_samples)
    L.check(lib.nc_sample_pdf(ctypes.byref(a), L.raw_stream(dev)), "nc_sample_pdf")
    return out.reshape(*lead, N_samples)
