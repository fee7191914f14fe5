"""torch.autograd.Function wrappers around libnicecore.so.

``NiceRenderFn``   = Renderer.render_batch_ray (src/utils/Renderer.py:95-262) forward +
                     autograd backward, in two C-ABI calls; optionally with the
                     Mapper / Tracker rendering loss fused in (a 4th output).
``NiceEvalFn``     = NICE.forward (src/conv_onet/models/decoder.py:336-370) on caller
                     points.

Tensors are handed over as raw device pointers + strides; the library enqueues on
the current HIP stream and never synchronises.  Gradients honour
``ctx.needs_input_grad``: grids / decoder parameters / rays that do not need a
gradient are not computed (the tracker's ray-only mode skips every weight
gradient and grid scatter).
"""
from __future__ import annotations

import ctypes
import operator
import os
import weakref

import torch

from . import _lib as L


def _ptr(t):
    return t.data_ptr() if t is not None else None


_data_ptr = torch.Tensor.data_ptr


_unflatten = torch._C._nn.unflatten_dense_tensors  # flat, tensors -> views shaped like tensors

_stream = L.raw_stream


def _bound_rows(b) -> list:
    """[[lo, hi]] * 3 as Python floats.  For a device-resident bound the rows are
    cached ON the tensor object, tagged with its storage pointer and version counter,
    so the per-call path never synchronises on a D2H copy.  (A cache keyed by
    data_ptr alone is wrong: the caching allocator hands freed addresses to new
    tensors.)"""
    if isinstance(b, torch.Tensor):
        tag = (b.data_ptr(), b._version)
        hit = getattr(b, "_nicecore_rows", None)
        if hit is not None and hit[0] == tag:
            return hit[1]
        t = b.detach().to("cpu", torch.float64).reshape(3, 2)
        rows = [[float(t[k, 0]), float(t[k, 1])] for k in range(3)]
        try:
            b._nicecore_rows = (tag, rows)
        except (AttributeError, RuntimeError):
            pass
        return rows
    t = torch.as_tensor(b, dtype=torch.float64).reshape(3, 2)
    return [[float(t[k, 0]), float(t[k, 1])] for k in range(3)]


def deterministic_requested(spec=None) -> bool:
    """NC_DETERMINISTIC (ordered grid-gradient reduction instead of float atomics):
    asked for by ``spec["deterministic"]``, else by the environment variable
    ``NC_DETERMINISTIC=1`` or ``torch.use_deterministic_algorithms(True)``."""
    d = spec.get("deterministic") if spec else None
    if d is not None:
        return bool(d)
    return os.environ.get("NC_DETERMINISTIC", "0") == "1" or torch.are_deterministic_algorithms_enabled()


# the forward zero-fills the backward's grid-gradient buffer (nc_render_args.grad_zero);
# NICECORE_FWD_ZERO=0 falls back to a separate fill in the backward (A/B timing)
_FWD_ZERO = os.environ.get("NICECORE_FWD_ZERO", "1") != "0"
# NICECORE_SAVE_JAC=1: the forward keeps the trilinear Jacobian for the coordinate gradient
# (NC_SAVE_POINT_JACOBIAN) instead of the backward re-reading the grid corners.  Off by
# default: measured at C2 it moves as much time into k_grid_gather (+6..12 us, 55 MB more
# writes) as it saves in k_mlp_dx (-6..7 us) -- BA 0.393 vs 0.399 ms, tracker 0.2065 vs
# 0.2076 ms per step (profiles/r01/jacobian_ab.txt)
_SAVE_JAC = os.environ.get("NICECORE_SAVE_JAC", "0") == "1"


def _flags(ctx, spec, coord_inputs=()):
    """NC_SAVE_FOR_BACKWARD when anything needs a gradient; NC_SAVE_POINT_JACOBIAN when
    the inputs at ``coord_inputs`` (rays / points) do; NC_DETERMINISTIC on request."""
    if not any(ctx.needs_input_grad):
        return 0
    f = L.NC_SAVE_FOR_BACKWARD | (L.NC_DETERMINISTIC if deterministic_requested(spec) else 0)
    if _SAVE_JAC and any(ctx.needs_input_grad[i] for i in coord_inputs):
        f |= L.NC_SAVE_POINT_JACOBIAN
    return f


def decoder_modules(decoders):
    return [getattr(decoders, n + "_decoder", None) for n in L.DECODER_NAMES]


def decoder_params(module, kind: int) -> list:
    """Parameters of one decoder in nn.Module.parameters() order (the flat-gradient
    order of the ABI)."""
    ps = []
    if kind != L.DEC_COARSE:
        for i in range(5):
            ps += [module.fc_c[i].weight, module.fc_c[i].bias]
        ps.append(module.embedder._B)
    for i in range(5):
        ps += [module.pts_linears[i].weight, module.pts_linears[i].bias]
    ps += [module.output_linear.weight, module.output_linear.bias]
    return ps


def _check_param(t, device):
    if t.device != device or t.dtype != torch.float32 or not t.is_contiguous():
        raise L.NiceCoreError(f"decoder parameters must be contiguous float32 on {device}")


def _fill_decoder(nd: L.NcDecoderParams, kind: int, params: list, bound, device):
    for t in params:
        _check_param(t, device)
    k = 0
    if kind != L.DEC_COARSE:
        for i in range(5):
            nd.fc_w[i] = params[k].data_ptr(); nd.fc_b[i] = params[k + 1].data_ptr(); k += 2
        nd.fourier_B = params[k].data_ptr(); k += 1
    for i in range(5):
        nd.lin_w[i] = params[k].data_ptr(); nd.lin_b[i] = params[k + 1].data_ptr(); k += 2
    nd.out_w = params[k].data_ptr(); nd.out_b = params[k + 1].data_ptr()
    nd.grad = None
    rows = _bound_rows(bound)
    for a in range(3):
        nd.bound[a][0], nd.bound[a][1] = rows[a]


def _fill_grid(ng: L.NcGrid, t, device):
    if t.dim() != 5 or t.shape[0] != 1 or t.shape[1] != 32:
        raise L.NiceCoreError(f"feature grid must be [1,32,D,H,W], got {tuple(t.shape)}")
    if t.dtype != torch.float32 or t.device != device:
        raise L.NiceCoreError(f"feature grid must be float32 on {device}")
    ng.data = t.data_ptr()
    ng.grad = None
    for a in range(3):
        ng.dims[a] = t.shape[2 + a]
    st = t.stride()
    for a in range(4):
        ng.stride[a] = st[1 + a]
        ng.grad_stride[a] = st[1 + a]


_NCGRID_BYTES = ctypes.sizeof(L.NcGrid)


def _fill_grid_cached(ng: L.NcGrid, t, device):
    """_fill_grid through an image cached ON the caller's grid tensor, tagged with its
    storage pointer, strides, shape, dtype and device (the per-call checks and ~15 ctypes
    field writes become one tag compare and one memmove)."""
    tag = (t.data_ptr(), t.stride(), t.shape, t.dtype, t.device)
    hit = getattr(t, "_nicecore_grid", None)
    if hit is None or hit[0] != tag:
        img = L.NcGrid()
        _fill_grid(img, t, device)
        hit = (tag, img)
        try:
            t._nicecore_grid = hit
        except (AttributeError, RuntimeError):
            pass
    elif t.device != device:
        raise L.NiceCoreError(f"feature grid must be float32 on {device}")
    ctypes.memmove(ctypes.addressof(ng), ctypes.addressof(hit[1]), _NCGRID_BYTES)


def _decoder_bound(module, name):
    b = getattr(module, "bound", None)
    if b is None:
        raise L.NiceCoreError(
            f"{name}_decoder.bound is not set (NICE_SLAM.load_bound assigns it, "
            "src/NICE_SLAM.py:202-208)")
    return b


def _fast_decoder_params(module, kind: int):
    """decoder_params() through the modules' own dicts (no ModuleList indexing):
    the per-call validation path.  Falls back to attribute access."""
    try:
        mm = module._modules
        ps = []
        if kind != L.DEC_COARSE:
            fc = mm["fc_c"]._modules
            for i in ("0", "1", "2", "3", "4"):
                q = fc[i]._parameters
                ps += [q["weight"], q["bias"]]
            emb = mm["embedder"]
            B = emb._parameters.get("_B")
            ps.append(B if B is not None else emb._B)
        pl = mm["pts_linears"]._modules
        for i in ("0", "1", "2", "3", "4"):
            q = pl[i]._parameters
            ps += [q["weight"], q["bias"]]
        q = mm["output_linear"]._parameters
        ps += [q["weight"], q["bias"]]
        return ps
    except (KeyError, AttributeError):
        return decoder_params(module, kind)


class _Plan:
    """Binding of one (decoders module, stage): which decoders / grids the stage
    touches, the decoder parameters in ABI order, and a pre-filled ctypes image of
    the decoder pointer tables.  Cached per decoders object (``make_plan``) and
    re-validated on every call by object identity + storage pointer + bound tag,
    so a replaced parameter, a ``.data`` swap or a new bound rebuilds it."""

    def __init__(self, stage: int, decoders):
        self.stage = stage
        self.decs = sorted(L.STAGE_DECODERS[stage])
        self.grids = L.STAGE_GRIDS[stage]
        mods = decoder_modules(decoders)
        self.modules = {k: mods[k] for k in self.decs}
        for k in self.decs:
            if self.modules[k] is None:
                raise L.NiceCoreError(f"stage needs the {L.DECODER_NAMES[k]} decoder")
        self.params = {k: decoder_params(self.modules[k], k) for k in self.decs}
        self.bounds = {k: _decoder_bound(self.modules[k], L.DECODER_NAMES[k]) for k in self.decs}
        self._flat = tuple(p for k in self.decs for p in self.params[k])
        sl, o = {}, 0
        for k in self.decs:
            sl[k] = (o, o + len(self.params[k]))
            o += len(self.params[k])
        self._slices = sl
        self._sig = None
        self._dec_img = None
        self._templates = {}
        self.grad_pool = {}  # _GradBuffer entries kept for reuse (see _GradBuffer)

    def flat_params(self):
        return list(self._flat)

    def param_slices(self):
        return self._slices

    def _signature(self):
        bt = []
        for k in self.decs:
            b = self.bounds[k]
            bt.append((b.data_ptr(), b._version) if isinstance(b, torch.Tensor) else id(b))
        return tuple(map(_data_ptr, self._flat)), tuple(bt)

    def still_valid(self, decoders) -> bool:
        mods = decoder_modules(decoders)
        for k in self.decs:
            m = mods[k]
            if m is not self.modules[k] or getattr(m, "bound", None) is not self.bounds[k]:
                return False
            cur = _fast_decoder_params(m, k)
            old = self.params[k]
            if len(cur) != len(old) or any(a is not b for a, b in zip(cur, old)):
                return False
        return True

    def decoder_image(self, device):
        """(NcDecoderParams * 4) with the pointers / bounds filled (grad = NULL)."""
        sig = self._signature()
        if sig != self._sig or self._dec_img is None:
            img = (L.NcDecoderParams * 4)()
            for k in self.decs:
                _fill_decoder(img[k], k, self.params[k], self.bounds[k], device)
            self._dec_img, self._sig = img, sig
            self._templates.clear()
        return self._dec_img

    def render_template(self, device, n_strat, n_surf, bound):
        """NcRenderArgs with every per-plan field filled; per call the caller copies
        it (from_buffer_copy) and sets the tensors."""
        img = self.decoder_image(device)
        bkey = (bound.data_ptr(), bound._version) if isinstance(bound, torch.Tensor) else id(bound)
        key = ("render", n_strat, n_surf, bkey)
        t = self._templates.get(key)
        if t is None:
            from .scene import linspace_tables
            ts, tsurf = linspace_tables(n_strat, n_surf)
            t = L.NcRenderArgs()
            t.abi_version = L.NC_ABI_VERSION
            t.stage = self.stage
            t.n_strat, t.n_surf = n_strat, n_surf
            rows = _bound_rows(bound)
            for k in range(3):
                t.bound[k][0], t.bound[k][1] = rows[k]
            for k, v in enumerate(ts.tolist()):
                t.t_strat[k] = v
            for k, v in enumerate(tsurf.tolist()):
                t.t_surf[k] = v
            ctypes.memmove(ctypes.addressof(t.dec), ctypes.addressof(img), ctypes.sizeof(img))
            self._templates[key] = t
        return t

    def points_template(self, device):
        img = self.decoder_image(device)
        t = self._templates.get("points")
        if t is None:
            t = L.NcPointsArgs()
            t.abi_version = L.NC_ABI_VERSION
            t.stage = self.stage
            ctypes.memmove(ctypes.addressof(t.dec), ctypes.addressof(img), ctypes.sizeof(img))
            self._templates["points"] = t
        return t


_PLANS = weakref.WeakKeyDictionary()  # decoders module -> {stage: _Plan}


def _dense_strides(g):
    """The grid's own strides when it is dense (contiguous or channels_last_3d, the
    layouts AccumulateGrad keeps), else contiguous strides: a strided view of a larger
    tensor gets a dense gradient of its own shape."""
    if g.is_contiguous(memory_format=torch.channels_last_3d) or g.is_contiguous():
        return g.stride()
    C, D, H, W = g.shape[1:]
    return (C * D * H * W, D * H * W, H * W, W, 1)


def _dense_needs(needs_grids, sparse):
    """needs_input_grad of the grids minus those whose gradient goes to sparse rows."""
    if sparse is None:
        return needs_grids
    return tuple(bool(n) and not sparse.covers(k) for k, n in enumerate(needs_grids))


def _bind_sparse(sparse, args, plan, n_points=None):
    """Point the grids that have sparse gradient rows at them (nicecore.sparse): the
    forward (n_points given) reserves room for its claims, the backward re-binds the
    current buffers (a later forward may have grown them)."""
    if sparse is None:
        return
    for k in plan.grids:
        if sparse.covers(k):
            if n_points is None:
                sparse.bind_backward(args.grids[k], k)
            else:
                sparse.bind_forward(args.grids[k], k, n_points)


_PARAM_COUNT = {}  # decoder kind -> nc_param_count (a constant of the library)


def _param_count(lib, k):
    n = _PARAM_COUNT.get(k)
    if n is None:
        n = _PARAM_COUNT[k] = int(lib.nc_param_count(k))
    return n


def _grad_sizes(lib, plan, needs_params, needs_grids, grids):
    sl = plan.param_slices()
    gk = [k for k in plan.grids if needs_grids[k]]
    pk = [k for k in plan.decs if any(needs_params[sl[k][0]:sl[k][1]])]
    gsize = sum(grids[k].numel() for k in gk)
    psize = {k: _param_count(lib, k) for k in pk}
    return gk, pk, gsize, psize


class _GradBuffer:
    """Every gradient of one backward call in ONE float32 buffer: the grid gradients
    first (strided views with each grid's own memory format, zero-filled by a single
    kernel), then one flat parameter vector per decoder whose parameters need a
    gradient (written, not accumulated, by the library), and the per-parameter
    views of those vectors.  The backward hands out detached aliases of the views:
    AccumulateGrad steals them as the leaves' .grad (their strides obey the layout
    contract) and distributed.allreduce_grads reduces the shared buffer with one
    collective.

    The buffer and its views are kept for reuse (``_grad_buffer``): once nothing
    outside the entry references its storage any more (the caller set the .grad of
    the last step to None, Mapper.py:620 / Tracker.py:135 ``zero_grad``), the next
    call takes the same buffer and views instead of building ~80 new views (the
    host cost of the drop-in path).  Entries are per (plan, stream, gradient set),
    so reuse is stream-ordered like the caching allocator's, and never used inside a
    stream capture (memory captured into a graph stays in the graph's pool).

    Stream contract: unlike the caching allocator the pool has no record_stream, so the
    .grad tensors must be consumed on the render stream or on a stream that the render
    stream waits on before the next forward (whose zero-fill rewrites a reused buffer).
    The library's own consumers obey it: torch.optim and torch.distributed's collectives
    (distributed.allreduce_grads / allreduce_rows_async: RCCL waits on the current stream
    before it reads, and ``work.wait()`` makes the current stream wait on RCCL before the
    caller goes on).  A caller that reads .grad on a user stream must make the render
    stream wait on that stream (``torch.cuda.current_stream().wait_stream(s)``) before
    the next render."""

    __slots__ = ("key", "buf", "gsize", "grid_grads", "flats", "pviews", "base")

    def __init__(self, key, plan, pk, gk, gsize, psize, grids, device):
        self.key, self.gsize = key, gsize
        self.buf = buf = torch.empty(gsize + sum(psize.values()), device=device, dtype=torch.float32)
        self.grid_grads = [None] * 4
        off = 0
        for k in gk:
            g = grids[k]
            self.grid_grads[k] = torch.as_strided(buf, g.shape, _dense_strides(g), off)
            off += g.numel()
        self.flats = {}
        self.pviews = []
        for k in plan.decs:
            ps = plan.params[k]
            if k in psize:
                self.flats[k] = f = buf[off:off + psize[k]]
                off += psize[k]
                self.pviews += _unflatten(f, ps)
            else:
                self.pviews += [None] * len(ps)
        self.base = _use_count(buf)

    def free(self):
        return _use_count(self.buf) == self.base

    def bind(self, args, plan, sparse):
        for k in plan.grids:
            args.grids[k].grad = None
            args.grids[k].grad_rows = None
        _bind_sparse(sparse, args, plan)
        for k, gg in enumerate(self.grid_grads):
            if gg is not None:
                args.grids[k].grad = gg.data_ptr()
                st = gg.stride()
                for ax in range(4):
                    args.grids[k].grad_stride[ax] = st[1 + ax]
        for k in plan.decs:
            args.dec[k].grad = None
        for k, f in self.flats.items():
            args.dec[k].grad = f.data_ptr()

    def outputs(self, needs_params):
        """(grid gradients, parameter gradients) as fresh aliases (None where not needed)."""
        gg = [g.detach() if g is not None else None for g in self.grid_grads]
        pg = [v.detach() if (v is not None and n) else None for v, n in zip(self.pviews, needs_params)]
        return gg, pg

    def zero(self):
        self.buf.zero_()


def _use_count(t):
    return torch._C._storage_Use_Count(t.untyped_storage()._cdata)


def _grad_buffer(lib, plan, needs_params, needs_grids, grids, device, stream):
    """The _GradBuffer for one backward call: a free pooled one with the same layout
    when there is one, else a new one.  Returns (entry, fresh)."""
    gk, pk, gsize, psize = _grad_sizes(lib, plan, needs_params, needs_grids, grids)
    if torch.cuda.is_current_stream_capturing():
        return _GradBuffer(None, plan, pk, gk, gsize, psize, grids, device), True
    key = (stream, tuple(gk), tuple(pk), tuple((grids[k].shape, _dense_strides(grids[k])) for k in gk))
    pool = plan.grad_pool
    e = pool.pop(key, None)
    if e is not None and e.free():
        return e, False
    return _GradBuffer(key, plan, pk, gk, gsize, psize, grids, device), True


def _release(plan, entry):
    if entry is not None and entry.key is not None:
        plan.grad_pool[entry.key] = entry


PARAM_GRAD_MODES = ("autograd", "direct")
# default for render_rays / render_rays_loss / Renderer when the caller does not choose
_PARAM_GRADS = os.environ.get("NICECORE_PARAM_GRADS", "direct")
_requires_grad = operator.attrgetter("requires_grad")
_ANCHORS = {}  # device -> zero-size leaf that connects a "direct" render to the graph


def param_inputs(spec, plan, device, mode=None):
    """The decoder-parameter inputs of NiceRenderFn.

    ``"direct"`` (default): the parameters stay out of the autograd graph and the
    backward writes their ``.grad`` itself -- set when None, added otherwise, the values
    AccumulateGrad would give (also when other terms of the loss reach the same
    parameters through autograd: whichever runs second adds).  One zero-size anchor
    leaf stands in for them, so ~80 AccumulateGrad nodes and Function inputs per call
    disappear from the host path; the reference's loops (loss.backward();
    optimizer.step(); optimizer.zero_grad(), Mapper.py:598-625, Tracker.py:113-135) see
    the same .grad.  A backward that does not reach the parameters -- torch.autograd.grad
    (loss, [camera]) as the Tracker's callers may write it, or backward(inputs=[...])
    without them -- is detected (the engine will not execute the anchor's
    AccumulateGrad node): the weight gradients are then neither computed (no k_mlp_dw)
    nor written, as autograd would leave them.  What it does not support: hooks on the
    decoder parameters, and torch.autograd.grad asked for the parameters themselves
    (their gradient goes to .grad, not to the returned tuple: use "autograd" for that).
    ``"autograd"`` (``rendering: {param_grads: autograd}`` in the config, or
    ``NICECORE_PARAM_GRADS=autograd``): the parameters themselves, so their gradients
    reach ``.grad`` through AccumulateGrad like any autograd leaf (hooks,
    autograd.grad and DDP see them), at ~0.3 ms more host time per call at C2."""
    mode = mode or _PARAM_GRADS
    if mode == "autograd":
        return plan._flat
    if mode != "direct":
        raise L.NiceCoreError(f"param_grads must be one of {PARAM_GRAD_MODES}, got {mode!r}")
    flat = plan._flat
    needs = tuple(map(_requires_grad, flat)) if torch.is_grad_enabled() else (False,) * len(flat)
    spec["param_needs"], spec["direct_params"] = needs, flat
    if not any(needs):
        return ()
    a = _ANCHORS.get(device)
    if a is None:
        a = _ANCHORS[device] = torch.empty(0, device=device, requires_grad=True)
    return (a,)


def _engine_reaches(anchor):
    """Whether the running backward will execute the direct-mode anchor's AccumulateGrad
    node, i.e. whether the decoder parameters are among the gradients it computes.  A
    torch without the query (a private engine API) is answered "yes": the parameters'
    .grad is written, the behaviour before the check existed."""
    try:
        node = torch.autograd.graph.get_gradient_edge(anchor).node
        return bool(torch._C._will_engine_execute_node(node))
    except (AttributeError, RuntimeError):
        return True


def _attach(pairs):
    """AccumulateGrad's effect for the direct mode: .grad set when None, else added."""
    for p, g in pairs:
        if p.grad is None:
            p.grad = g
        else:
            p.grad.add_(g)


def _versions(params):
    return tuple(p._version if isinstance(p, torch.Tensor) else None for p in params)


def _check_versions(params, versions):
    """The backward reads the decoder weights the forward used (k_mlp_dx's weight image is
    built by the forward, nc_wimage.h), as the reference's nn.Linear saves its weight for
    backward: a parameter changed in place in between is an error there, and here."""
    for p, v in zip(params, versions):
        if isinstance(p, torch.Tensor) and p._version != v:
            raise RuntimeError("one of the variables needed for gradient computation has been modified by an "
                               "inplace operation: a decoder parameter changed between the nicecore forward "
                               "and its backward")


class NiceRenderFn(torch.autograd.Function):
    """render_batch_ray on the HIP core.  Inputs: (spec, rays_o, rays_d, gt_depth|None,
    grid_coarse|None, grid_middle|None, grid_fine|None, grid_color|None, *params).
    Outputs (depth, var, color), plus the float64 scalar loss when ``spec["loss"]`` =
    (kind, flags, w_color, target_depth, target_color|None) asks for one (targets
    are data: no gradient flows to them, as in the reference)."""

    @staticmethod
    def forward(ctx, spec, rays_o, rays_d, gt_depth, g0, g1, g2, g3, *params):
        lib = L.load()
        plan = spec["plan"]
        sparse = spec.get("sparse")
        device = rays_o.device
        if device.type != "cuda":
            raise L.NiceCoreError("nicecore renders on a HIP device; tensors are on " + str(device))
        ctx.set_materialize_grads(False)  # unused outputs: NULL upstream gradient, no zero fill
        rays_o = rays_o.detach().float().contiguous()
        rays_d = rays_d.detach().float().contiguous()
        N = rays_o.shape[0]
        a = L.NcRenderArgs.from_buffer_copy(
            plan.render_template(device, spec["n_strat"], spec["n_surf"], spec["bound"]))
        a.flags = _flags(ctx, spec, (1, 2))
        pneeds = spec.get("param_needs")  # "direct" parameter gradients (param_inputs)
        ctx.direct = pneeds is not None
        ctx.n_param_inputs = len(params)
        ctx.anchor = params[0] if (ctx.direct and params) else None
        if pneeds is None:
            pneeds = ctx.needs_input_grad[8:]
        else:
            params = spec["direct_params"]
        ctx.pneeds = pneeds
        if a.flags & L.NC_SAVE_FOR_BACKWARD:  # decoders without a weight gradient: no activation records
            sl = plan.param_slices()
            for k in plan.decs:
                if not any(pneeds[sl[k][0]:sl[k][1]]):
                    a.flags |= L.NC_NO_WEIGHT_GRAD(k)
        a.n_rays = N
        a.rays_o = rays_o.data_ptr()
        a.rays_d = rays_d.data_ptr()
        gt = None
        if gt_depth is not None:
            gt = gt_depth.detach().reshape(-1).float().contiguous()
            a.gt_depth = gt.data_ptr()
        dmax = spec.get("depth_max")
        if dmax is not None:
            dmax = dmax.detach().reshape(1).float().contiguous()
            a.depth_max = dmax.data_ptr()
        # hierarchical sampling (Renderer.py:239-259): pass 1 reports its depths and
        # weights, pass 2 merges the sample_pdf depths (no gradient) into its samples
        zx = spec.get("z_extra")
        if zx is not None:
            zx = zx.detach().double().contiguous()
            a.z_extra, a.n_extra = zx.data_ptr(), zx.shape[-1]
        for name in ("z_out", "weights_out"):
            t = spec.get(name)
            if t is not None:
                setattr(a, name, t.data_ptr())
        # stratified sampling options (Renderer.py:208-219): lindisp, perturb's draws
        a.lindisp = 1 if spec.get("lindisp") else 0
        tr = spec.get("t_rand")
        if tr is not None:
            if tr.dtype != torch.float32 or not tr.is_contiguous() or tuple(tr.shape) != (N, spec["n_strat"]) \
                    or tr.device != device:
                raise L.NiceCoreError("t_rand must be a contiguous float32 [N, n_strat] tensor on the render device")
            a.t_rand = tr.data_ptr()
        # the callers' bbox pre-filter as a per-ray mask (ABI v10 ray_valid): dropped rays are
        # out of the batch depth max, the loss and every gradient -- no compaction, no host sync
        rv = spec.get("ray_valid")
        if rv is not None:
            rv = rv.detach().reshape(-1)
            if rv.shape[0] != N or rv.device != device:
                raise L.NiceCoreError("ray_mask must hold one entry per ray, on the render device")
            rv = (rv.view(torch.uint8) if rv.dtype == torch.bool else rv.to(torch.uint8)).contiguous()
            a.ray_valid = rv.data_ptr()
        grids = (g0, g1, g2, g3)
        gkeep = []
        for k in plan.grids:
            if grids[k] is None:
                raise L.NiceCoreError(f"stage needs {L.GRID_KEYS[k]}")
            _fill_grid_cached(a.grids[k], grids[k], device)
            gkeep.append(grids[k].detach())
        if a.flags & L.NC_SAVE_FOR_BACKWARD:
            _bind_sparse(sparse, a, plan, N * (spec["n_strat"] + spec["n_surf"] + a.n_extra))
        depth = torch.empty(N, device=device, dtype=torch.float64)
        var = torch.empty(N, device=device, dtype=torch.float64)
        color = torch.empty(N, 3, device=device, dtype=torch.float32)
        a.depth, a.var, a.color = depth.data_ptr(), var.data_ptr(), color.data_ptr()
        loss_spec = spec.get("loss")
        loss = tgt = None
        if loss_spec is not None:
            kind, lflags, w, tdepth, tcolor = loss_spec
            tgt = (tdepth.detach().reshape(-1).float().contiguous(),
                   tcolor.detach().reshape(-1, 3).float().contiguous() if tcolor is not None else None)
            if tgt[0].shape[0] != N or (tgt[1] is not None and tgt[1].shape[0] != N):
                raise L.NiceCoreError("loss targets must have one row per ray")
            loss = torch.empty((), device=device, dtype=torch.float64)
            a.loss, a.loss_flags, a.w_color = kind, lflags, float(w)
            a.loss_depth, a.loss_color, a.loss_out = tgt[0].data_ptr(), _ptr(tgt[1]), loss.data_ptr()
        # the backward's gradient buffer: taken here and its grid part zero-filled by the
        # forward's gather kernel (no separate fill launch); used by the first backward call
        ctx.grad_entry = None
        stream = _stream(device)
        dneeds = _dense_needs(ctx.needs_input_grad[4:8], sparse)
        if _FWD_ZERO and any(dneeds):
            e, _ = _grad_buffer(lib, plan, pneeds, dneeds, grids, device, stream)
            if e.gsize:
                ctx.grad_entry = e
                a.grad_zero, a.grad_zero_floats = e.buf.data_ptr(), e.gsize
            else:
                _release(plan, e)
        nbytes = lib.nc_render_workspace_bytes(ctypes.byref(a))
        if nbytes == 0:
            L.check(-1, "nc_render_workspace_bytes")
        ws = torch.empty(nbytes, device=device, dtype=torch.uint8)
        L.check(lib.nc_render_forward(ctypes.byref(a), ws.data_ptr(), nbytes, stream), "nc_render_forward")
        a.grad_zero, a.grad_zero_floats = None, 0
        ctx.args, ctx.ws, ctx.nbytes, ctx.plan = a, ws, nbytes, plan
        ctx.sparse = sparse
        ctx.defer = spec.get("defer")
        ctx.keep = (rays_o, rays_d, gt, dmax, gkeep, params, tgt, zx, tr, rv)
        ctx.pversions = _versions(params)
        a.z_out, a.weights_out = None, None  # pass-1 outputs: not rewritten by the backward
        ctx.grids = grids
        if loss is None:
            return depth, var, color
        return depth, var, color, loss

    @staticmethod
    def backward(ctx, g_depth, g_var, g_color, g_loss=None):
        _check_versions(ctx.keep[5], ctx.pversions)
        lib = L.load()
        a, plan = ctx.args, ctx.plan
        need = ctx.needs_input_grad
        rays_o = ctx.keep[0]
        device = rays_o.device
        gd = g_depth.detach().double().contiguous() if g_depth is not None else None
        gv = g_var.detach().double().contiguous() if g_var is not None else None
        gc = g_color.detach().float().contiguous() if g_color is not None else None
        a.g_depth, a.g_var, a.g_color = _ptr(gd), _ptr(gv), _ptr(gc)
        gl = g_loss.detach().double().reshape(1).contiguous() if g_loss is not None else None
        a.g_loss = _ptr(gl)
        g_ro = torch.empty_like(rays_o) if need[1] else None
        g_rd = torch.empty_like(rays_o) if need[2] else None
        # the kernel computes d rays_o and d rays_d together; ask for both if either is needed
        if (g_ro is None) != (g_rd is None):
            g_ro = g_ro if g_ro is not None else torch.empty_like(rays_o)
            g_rd = g_rd if g_rd is not None else torch.empty_like(rays_o)
        a.g_rays_o, a.g_rays_d = _ptr(g_ro), _ptr(g_rd)
        needs_params = ctx.pneeds
        skip_params = ctx.anchor is not None and not _engine_reaches(ctx.anchor)
        if skip_params:  # autograd.grad / backward(inputs=) without the decoder parameters
            needs_params = (False,) * len(needs_params)
        stream = _stream(device)
        e = ctx.grad_entry
        ctx.grad_entry = None  # a second backward (retain_graph) gets a fresh, zeroed buffer
        if e is None:
            e, _ = _grad_buffer(lib, plan, needs_params, _dense_needs(need[4:8], ctx.sparse), ctx.grids,
                                device, stream)
            if e.gsize:
                e.buf[:e.gsize].zero_()
        e.bind(a, plan, ctx.sparse)
        if skip_params:
            for k in plan.decs:
                a.dec[k].grad = None  # NULL decoder gradient: the library skips k_mlp_dw
        if rays_o.shape[0] == 0:  # empty batch: nothing is launched, every gradient is zero
            e.zero()
            grid_grads, pg = e.outputs(needs_params)
            _release(plan, e)
            return (None, g_ro if need[1] else None, g_rd if need[2] else None, None, *grid_grads,
                    *NiceRenderFn._param_outputs(ctx, pg))
        defer = ctx.defer if any(needs_params) else None
        if defer is not None:
            a.flags |= L.NC_DEFER_PARAM_GRADS
        try:
            L.check(lib.nc_render_backward(ctypes.byref(a), ctx.ws.data_ptr(), ctx.nbytes, stream),
                    "nc_render_backward")
        finally:
            a.flags &= ~L.NC_DEFER_PARAM_GRADS
        grid_grads, pg = e.outputs(needs_params)
        if defer is not None:  # weight gradients: launched and attached by defer.run()
            defer._add(L.NcRenderArgs.from_buffer_copy(a), ctx.ws, ctx.nbytes, e.flats,
                       [(p, g) for p, g in zip(ctx.keep[5], pg) if g is not None])
            pg = [None] * len(pg)
        _release(plan, e)
        return (None, g_ro if need[1] else None, g_rd if need[2] else None, None, *grid_grads,
                *NiceRenderFn._param_outputs(ctx, pg))

    @staticmethod
    def _param_outputs(ctx, pg):
        """The gradients returned for the parameter inputs: the parameters' own, or in
        the direct mode None for the anchor after attaching them to .grad here."""
        if not ctx.direct:
            return pg
        _attach([(p, g) for p, g in zip(ctx.keep[5], pg) if g is not None])
        return [None] * ctx.n_param_inputs


class DeferParamGrads:
    """Split a render backward in two so that a data-parallel caller can start the
    grid-gradient all-reduce while the decoder weight gradients are still being
    computed (the grid gradients are final after k_mlp_dx; k_mlp_dw comes after it).

    Pass it as ``defer_param_grads=`` to the render call; ``backward()`` then produces
    the grid and ray gradients only (NC_DEFER_PARAM_GRADS) and leaves the decoder
    parameters' ``.grad`` untouched; ``run()`` launches the weight gradients
    (nc_render_backward_params) of every backward since ``clear()`` and attaches them
    to the parameters (set when ``.grad`` is None, accumulated otherwise).  Both halves
    are graph-capturable (two nicecore.graph.GraphedStep captures, bench.py N > 1)."""

    def __init__(self):
        self.pending = []

    def clear(self):
        self.pending = []

    def _add(self, args, ws, nbytes, flats, pairs):
        self.pending.append((args, ws, nbytes, flats, pairs))

    def run(self):
        lib = L.load()
        for args, ws, nbytes, _flats, pairs in self.pending:
            stream = _stream(ws.device)
            L.check(lib.nc_render_backward_params(ctypes.byref(args), ws.data_ptr(), nbytes, stream),
                    "nc_render_backward_params")
            for p, g in pairs:
                if p.grad is None:
                    p.grad = g
                elif p.grad.data_ptr() != g.data_ptr():
                    p.grad.add_(g)


class NiceEvalFn(torch.autograd.Function):
    """NICE.forward(p, c_grid, stage) on the HIP core.  Inputs: (spec, p, g0..g3, *params)."""

    @staticmethod
    def forward(ctx, spec, p, g0, g1, g2, g3, *params):
        lib = L.load()
        plan = spec["plan"]
        sparse = spec.get("sparse")
        device = p.device
        if device.type != "cuda":
            raise L.NiceCoreError("nicecore evaluates on a HIP device; points are on " + str(device))
        pts = p.detach().reshape(-1, 3).double().contiguous()
        P = pts.shape[0]
        a = L.NcPointsArgs.from_buffer_copy(plan.points_template(device))
        a.n_points = P
        a.flags = _flags(ctx, spec, (1,))
        a.pts = pts.data_ptr()
        grids = (g0, g1, g2, g3)
        gkeep = []
        for k in plan.grids:
            if grids[k] is None:
                raise L.NiceCoreError(f"stage needs {L.GRID_KEYS[k]}")
            _fill_grid_cached(a.grids[k], grids[k], device)
            gkeep.append(grids[k].detach())
        if a.flags & L.NC_SAVE_FOR_BACKWARD:
            _bind_sparse(sparse, a, plan, P)
        raw = torch.empty(P, 4, device=device, dtype=torch.float32)
        a.raw = raw.data_ptr()
        nbytes = lib.nc_points_workspace_bytes(ctypes.byref(a))
        ws = torch.empty(max(nbytes, 1), device=device, dtype=torch.uint8)
        stream = _stream(device)
        L.check(lib.nc_points_forward(ctypes.byref(a), ws.data_ptr(), nbytes, stream), "nc_points_forward")
        ctx.args, ctx.ws, ctx.nbytes, ctx.plan = a, ws, nbytes, plan
        ctx.sparse = sparse
        ctx.keep = (pts, gkeep, params)
        ctx.pversions = _versions(params)
        ctx.grids = grids
        ctx.p_dtype, ctx.p_shape = p.dtype, p.shape
        return raw

    @staticmethod
    def backward(ctx, g_raw):
        _check_versions(ctx.keep[2], ctx.pversions)
        lib = L.load()
        a, plan = ctx.args, ctx.plan
        need = ctx.needs_input_grad
        pts = ctx.keep[0]
        device = pts.device
        gr = g_raw.detach().float().contiguous()
        a.g_raw = gr.data_ptr()
        g_pts = torch.empty_like(pts) if need[1] else None
        a.g_pts = _ptr(g_pts)
        needs_params = need[6:]
        stream = _stream(device)
        e, _ = _grad_buffer(lib, plan, needs_params, _dense_needs(need[2:6], ctx.sparse), ctx.grids, device, stream)
        if e.gsize:
            e.buf[:e.gsize].zero_()
        e.bind(a, plan, ctx.sparse)
        if a.n_points == 0:  # no points: nothing is launched, every gradient is zero
            e.zero()
        else:
            L.check(lib.nc_points_backward(ctypes.byref(a), ctx.ws.data_ptr(), ctx.nbytes, stream),
                    "nc_points_backward")
        grid_grads, pg = e.outputs(needs_params)
        _release(plan, e)
        gp = g_pts.to(ctx.p_dtype).reshape(ctx.p_shape) if g_pts is not None else None
        return (None, gp, *grid_grads, *pg)


def make_plan(stage, decoders) -> _Plan:
    s = L.STAGES[stage] if isinstance(stage, str) else int(stage)
    try:
        per = _PLANS.get(decoders)
    except TypeError:  # not weak-referenceable: no caching
        return _Plan(s, decoders)
    if per is None:
        per = {}
        _PLANS[decoders] = per
    plan = per.get(s)
    if plan is None or not plan.still_valid(decoders):
        plan = _Plan(s, decoders)
        per[s] = plan
    return plan
