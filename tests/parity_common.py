"""Shared setup for GPU parity runs: build the drop-in Renderer + NICE on a HIP
device from the golden scene, render a golden case, back-propagate the stored
upstream gradients and collect every output / input gradient."""
from __future__ import annotations

import types

import numpy as np
import torch

from conftest import load_case, load_initstd_meta, load_meta, load_scene
from nicecore import decoder as D
from nicecore import scene as S
from nicecore.renderer import Renderer

CFG = {"rendering": dict(S.DEFAULT_RENDERING), "scale": 1, "occupancy": True}


def build_model(params, bound, cbound, device):
    m = D.build_default_nice(seed=0)
    m.load_state_dict(params)
    m = m.to(device)
    b = bound.to(device)
    m.bound = b
    for n in ("middle", "fine", "color"):
        getattr(m, n + "_decoder").bound = b
    m.coarse_decoder.bound = cbound.to(device)
    return m


def make_renderer(bound, H=48, W=64):
    slam = types.SimpleNamespace(nice=True, bound=bound, H=H, W=W, fx=40.0, fy=40.0, cx=31.5, cy=23.5)
    return Renderer(CFG, None, slam)


def case_stage(name):
    cases = load_meta()["cases"] + load_initstd_meta()["cases"]
    c = next(c for c in cases if c["name"] == name)
    return c["stage"], c["with_depth"]


def scene_of(name):
    """Golden scene a case was rendered on (make_golden.py / make_golden_initstd.py)."""
    return "initstd" if name.startswith("initstd_") else "tiny"


def run_case(name, device="cuda", channels_last=False, want=("rays", "grids", "params")):
    bound, cbound, grids, params = load_scene(scene_of(name))
    rec = load_case(name)
    stage, with_depth = case_stage(name)
    model = build_model(params, bound, cbound, device)
    for p in model.parameters():
        p.requires_grad_("params" in want)
    g = {}
    for k, v in grids.items():
        t = v.to(device)
        if channels_last:
            t = t.contiguous(memory_format=torch.channels_last_3d)
        g[k] = t.requires_grad_("grids" in want)
    ro = rec["rays_o"].to(device).requires_grad_("rays" in want)
    rd = rec["rays_d"].to(device).requires_grad_("rays" in want)
    gt = rec["gt_depth"].to(device) if with_depth else None
    r = make_renderer(bound)
    depth, var, color = r.render_batch_ray(g, model, rd, ro, device, stage, gt)
    torch.autograd.backward([depth, var, color],
                            [rec["g_depth"].to(device), rec["g_var"].to(device), rec["g_color"].to(device)])
    got = {"depth": depth.detach(), "var": var.detach(), "color": color.detach()}
    if "rays" in want:
        got["grad/rays_o"] = ro.grad
        got["grad/rays_d"] = rd.grad
    if "grids" in want:
        for k, v in g.items():
            if v.grad is not None:
                got["grad/" + k] = v.grad
    if "params" in want:
        for n, p in model.named_parameters():
            if p.grad is not None:
                got["grad/param/" + n] = p.grad
    return rec, {k: v.detach().cpu() for k, v in got.items()}


def hip_render_grads(grids, params, bound, cbound, ro, rd, stage, gt, upstream, channels_last=True,
                     make=None):
    """The HIP render + backward of given inputs (the drop-in Renderer, grids on the GPU in
    the chosen layout), upstream gradients ``upstream`` = (d depth, d var, d color); returns
    {name: cpu tensor} like run_case."""
    model = build_model(params, bound, cbound, "cuda")
    g = {}
    for k, v in grids.items():
        t = v.cuda()
        if channels_last:
            t = t.contiguous(memory_format=torch.channels_last_3d)
        g[k] = t.requires_grad_(True)
    ro_g, rd_g = ro.cuda().requires_grad_(True), rd.cuda().requires_grad_(True)
    r = (make or make_renderer)(bound)
    d, v, c = r.render_batch_ray(g, model, rd_g, ro_g, "cuda", stage, gt.cuda() if gt is not None else None)
    torch.autograd.backward([d, v, c], [t.cuda() for t in upstream])
    got = {"depth": d.detach(), "var": v.detach(), "color": c.detach(), "grad/rays_o": ro_g.grad,
           "grad/rays_d": rd_g.grad}
    for k, t in g.items():
        if t.grad is not None:
            got["grad/" + k] = t.grad
    for n, p in model.named_parameters():
        if p.grad is not None:
            got["grad/param/" + n] = p.grad
    return {k: t.detach().cpu() for k, t in got.items()}


def rel_err(got, ref):
    """max |got - ref| / max(|ref|_max, tiny) — scale-aware error of a whole tensor."""
    got = got.double().reshape(-1)
    ref = ref.double().reshape(-1)
    scale = float(ref.abs().max()) if ref.numel() else 0.0
    return float((got - ref).abs().max()) / max(scale, 1e-30) if ref.numel() else 0.0


def compare(rec, got):
    out = {}
    for k, v in got.items():
        if k in rec:
            out[k] = rel_err(v, rec[k])
        else:
            out[k] = float(v.abs().max())  # reference has no gradient here -> must be ~0
    return out


def oracle_render_grads(grids, params, dec_b, bound, ro, rd, stage, gt, upstream, f64=False, depth_max=None,
                        round_inputs=False, order=None):
    """CPU oracle render + backward; with f64=True everything runs in float64
    (ground truth; ``round_inputs``: keeping the reference's float32 input roundings,
    nice_oracle.float64_mode).  ``depth_max``: the batch-global max(gt_depth) of a sharded
    batch.  ``order``: a permutation the rays are rendered in (results un-permuted): the
    same float32 program with other summation orders.  Returns {name: tensor} like run_case."""
    from oracle import nice_oracle as O
    if order is not None:
        inv = torch.argsort(order)
        gd, gv, gc = upstream
        out = oracle_render_grads(grids, params, dec_b, bound, ro[order], rd[order], stage,
                                  gt[order] if gt is not None else None, (gd[order], gv[order], gc[order]),
                                  f64, depth_max, round_inputs)
        for k in ("depth", "var", "color", "grad/rays_o", "grad/rays_d"):
            out[k] = out[k][inv]
        return out
    cast = (lambda t: t.double()) if f64 else (lambda t: t)
    ro_c = cast(ro.clone()).requires_grad_(True)
    rd_c = cast(rd.clone()).requires_grad_(True)
    g_c = {k: cast(v.clone()).requires_grad_(True) for k, v in grids.items()}
    prm_c = {k: cast(v.clone()).requires_grad_(True) for k, v in params.items()}
    gt_c = cast(gt) if gt is not None else None
    ctx = O.float64_mode(round_inputs) if f64 else _null()
    with ctx:
        dm = None if depth_max is None else cast(depth_max.reshape(()).clone())
        d, v, c = O.render_batch_ray(g_c, prm_c, dec_b, bound, rd_c, ro_c, stage, gt_c, depth_max=dm)
        gd, gv, gc = upstream
        torch.autograd.backward([d, v, c], [gd, gv, cast(gc)])
    out = {"depth": d.detach(), "var": v.detach(), "color": c.detach(),
           "grad/rays_o": ro_c.grad, "grad/rays_d": rd_c.grad}
    for k, t in g_c.items():
        if t.grad is not None and float(t.grad.abs().max()) > 0:
            out["grad/" + k] = t.grad
    for k, t in prm_c.items():
        if t.grad is not None and float(t.grad.abs().max()) > 0:
            out["grad/param/" + k] = t.grad
    return out


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def score_vs_truth(got, ref32, ref64, out_floor=2e-5, grad_floor=2e-4):
    """{name: (err_hip, err_ref32, allowed)} where err = scale-aware error vs float64."""
    res = {}
    for k, t64 in ref64.items():
        if k not in got:
            res[k] = (float("inf"), 0.0, 0.0)
            continue
        e_hip = rel_err(got[k], t64)
        e_ref = rel_err(ref32[k], t64) if k in ref32 else 0.0
        floor = grad_floor if k.startswith("grad/") else out_floor
        res[k] = (e_hip, e_ref, max(4.0 * e_ref, floor))
    return res


# --- per-element parity ---------------------------------------------
# The per-tensor metric above (max error / max |ref|) cannot see a wrong value on a
# lightly-touched voxel or a low-weight ray while it stays below 2e-4 of the tensor's
# maximum.  The per-element gate, for every element e of every output and gradient:
#     |hip_e - t_e| <= ELEM_FACTOR * max_k |ref_k,e - t_e| + ELEM_FACTOR * rms_e(ref_0 - t)
# t: the oracle in float64 with the reference's float32 input roundings (p.float(), the
#    float32 lookup coordinates: nice_oracle.float64_mode(round_inputs=True)), i.e. the exact
#    value of the reference's float32 program;
# ref_k: float32 computations of the same program -- ref_0 the reference's own vectors
#    (golden cases) or the float32 oracle, ref_1, ref_2 the float32 oracle on the network with
#    its hidden units, Fourier features and grid channels permuted (permuted_problem: the same
#    function with every dot product summed in another order, as any other float32
#    implementation sums it; gradients mapped back);
# the floor: 4x the reference's own RMS float32 error over the tensor's non-zero elements -- below 1e-6 of the
#    tensor's max for the large tensors, above it where float32 itself is that far off (the
#    reference's own max error reaches 5.6e-6 of max on the golden decoder gradients).
# Grid gradients must also have the support of ref_0: the same voxels non-zero.
ELEM_FACTOR = 4.0


def elementwise_vs_truth(got, refs, truth, factor=ELEM_FACTOR):
    """{name: stats} over the tensors of ``truth``; ``refs``: one float32 reference dict or a
    list of them (the first one sets the floor and the support).  ``worst`` = max over
    elements of |hip - t| / allowed (<= 1 passes), ``n_bad`` elements above 1, relative L2
    errors ``l2_hip`` / ``l2_ref`` = ||x - t|| / ||t||, max-normalised errors ``max_hip`` /
    ``max_ref`` and the floor in units of the tensor's max, ``floor``."""
    refs = refs if isinstance(refs, (list, tuple)) else [refs]
    res = {}
    for k, t64 in truth.items():
        if k not in got or any(k not in r for r in refs):
            res[k] = {"worst": float("inf"), "n_bad": -1, "n": 0, "missing": True}
            continue
        t = t64.double().reshape(-1)
        if not t.numel():
            res[k] = {"worst": 0.0, "n_bad": 0, "n": 0}
            continue
        h = got[k].double().reshape(-1)
        ers = [(r[k].double().reshape(-1) - t).abs() for r in refs]
        er = torch.stack(ers).amax(0)
        scale = max(float(t.abs().max()), 1e-300)
        live = t != 0  # the RMS over the elements the reference computes (an untouched voxel's
        #                zero gradient is exact in every implementation and would dilute it)
        floor = factor * float(ers[0][live].pow(2).mean().sqrt()) if bool(live.any()) else 0.0
        eh = (h - t).abs()
        ratio = eh / (factor * er + max(floor, 1e-300))
        nt = float(t.norm()) or 1e-300
        res[k] = {"worst": float(ratio.max()), "n_bad": int((ratio > 1).sum()), "n": int(t.numel()),
                  "l2_hip": float(eh.norm()) / nt, "l2_ref": float(ers[0].norm()) / nt,
                  "max_hip": float(eh.max()) / scale, "max_ref": float(ers[0].max()) / scale,
                  "floor": floor / scale}
        if k.startswith("grad/grid_"):
            res[k]["support"] = grid_support_diff(got[k], refs[0][k])
    return res


def grid_support_diff(got, ref, tol=2.0 ** -24):
    """(voxels with a non-zero gradient only in ``got``, only in ``ref``, the largest such
    voxel's magnitude in units of max |ref|) of [1, C, D, H, W] grid gradients: a dropped or
    mis-addressed scatter shows here.  A voxel counts when its magnitude (max over channels)
    exceeds ``tol`` x max |ref| -- below float32's resolution at the tensor's scale a
    contribution is the product of an underflowing transmittance (T = prod (1 - alpha)
    reaches the float32 subnormals behind a surface; where it flushes to zero depends on
    the order of the product), not an addressing decision.  ``ref`` must make the same
    float32 corner decisions (the float32 reference, not a float64 truth: a coordinate
    within an ulp of a voxel plane picks other corners in float64)."""
    a = got.reshape(got.shape[-4], -1).abs().amax(0).double()
    b = ref.reshape(ref.shape[-4], -1).abs().amax(0).double()
    cut = tol * max(float(b.max()), 1e-300)
    only_a, only_b = (a != 0) & (b == 0), (b != 0) & (a == 0)
    mag = max(float(a[only_a].max()) if bool(only_a.any()) else 0.0,
              float(b[only_b].max()) if bool(only_b.any()) else 0.0) / max(float(b.max()), 1e-300)
    return int((only_a & (a > cut)).sum()), int((only_b & (b > cut)).sum()), mag, \
        int(only_a.sum()), int(only_b.sum())


def report_elementwise(title, res):
    """Print the per-tensor table (worst per-element ratio first) and return the failures."""
    print(f"\n[{title}] per-element vs float64 truth (worst ratio <= 1 passes; rel-L2 and max-normalised "
          f"errors hip / ref32; floor in units of max)")
    bad = {}
    for k, v in sorted(res.items(), key=lambda kv: -kv[1]["worst"]):
        sup = v.get("support")
        print(f"  {k:44s} worst {v['worst']:.3g}  n_bad {v['n_bad']}/{v['n']}  "
              f"l2 {v.get('l2_hip', float('nan')):.2e} / {v.get('l2_ref', float('nan')):.2e}  "
              f"max {v.get('max_hip', float('nan')):.2e} / {v.get('max_ref', float('nan')):.2e}  "
              f"floor {v.get('floor', float('nan')):.1e}"
              + (f"  support +{sup[0]} -{sup[1]} (below tol: +{sup[3] - sup[0]} -{sup[4] - sup[1]}, "
                 f"largest {sup[2]:.1e} of max)" if sup else ""))
        if not v["worst"] <= 1.0 or (sup and sup[:2] != (0, 0)):
            bad[k] = v
    worst = max((v["worst"] for v in res.values()), default=0.0)
    print(f"  worst per-element ratio over all tensors: {worst:.4g}")
    return bad


def collect_step(grids, model, ro, rd, outs=None, loss=None):
    """{name: cpu tensor} of a rendered step: outputs (when given) and every non-zero
    leaf gradient, in the oracle's naming."""
    got = {}
    if outs is not None:
        d, u, c = outs
        got.update({"depth": d.detach().cpu(), "var": u.detach().cpu(), "color": c.detach().cpu()})
    if loss is not None:
        got["loss"] = loss.detach().cpu().reshape(1)
    got["grad/rays_o"], got["grad/rays_d"] = ro.grad.detach().cpu(), rd.grad.detach().cpu()
    for k, g in grids.items():
        if g.grad is not None and float(g.grad.abs().max()) > 0:
            got["grad/" + k] = g.grad.detach().cpu()
    for n, p in model.named_parameters():
        if p.grad is not None and float(p.grad.abs().max()) > 0:
            got["grad/param/" + n] = p.grad.detach().cpu()
    return got


def oracle_mapper_refs(w, kw, stage="color", forms=((False, False, None), (True, False, None))):
    """The oracle's render + Mapper loss (Mapper.py:603-612) + backward on a bench workload
    ``w`` (bench.build_workload).  ``forms``: (float64, round_inputs, order[, perm_seed]) per
    result -- float32 / float64 computations, the float64 one with the reference's float32
    input roundings, the rays in another order (outputs and ray gradients un-permuted), or
    (perm_seed) the unit-permuted network (permuted_problem, gradients mapped back).
    Returns {form: {name: tensor}}; the default forms give {(False, False, None): ref32,
    (True, False, None): ref64}, also reachable as [False] / [True]."""
    from nicecore import scene as S
    from oracle import nice_oracle as O
    g_cpu0 = {k: v.detach().cpu().contiguous() for k, v in w["grids"].items()}
    prm0 = {n: p.detach().cpu() for n, p in w["model"].named_parameters()}
    ro0, rd0, gt0, gtc0 = (t.detach().cpu() for t in (w["ro"], w["rd"], w["gt"], w["gtc"]))
    dec_b = S.decoder_bounds(w["sc"].bound)
    refs = {}
    for form in forms:
        f64, rnd, order = form[:3]
        seed = form[3] if len(form) > 3 else None
        g_cpu, prm, un = (g_cpu0, prm0, None) if seed is None else permuted_problem(g_cpu0, prm0, seed)
        ro, rd, gt, gtc = (t if order is None else t[order] for t in (ro0, rd0, gt0, gtc0))
        cast = (lambda t: t.double()) if f64 else (lambda t: t)
        ro_c, rd_c = cast(ro.clone()).requires_grad_(True), cast(rd.clone()).requires_grad_(True)
        g_c = {k: cast(v.clone()).requires_grad_(True) for k, v in g_cpu.items()}
        p_c = {k: cast(v.clone()).requires_grad_(True) for k, v in prm.items()}
        with (O.float64_mode(rnd) if f64 else _null()):
            dd, uu, cc = O.render_batch_ray(g_c, p_c, dec_b, w["sc"].bound, rd_c, ro_c, stage, cast(gt))
            lo = O.mapper_loss(dd, cc, cast(gt), cast(gtc), kw["w_color_loss"], kw["color_term"])
            lo.backward()
        r = {"depth": dd.detach(), "var": uu.detach(), "color": cc.detach(), "loss": lo.detach().reshape(1),
             "grad/rays_o": ro_c.grad, "grad/rays_d": rd_c.grad}
        if order is not None:
            inv = torch.argsort(order)
            for k in ("depth", "var", "color", "grad/rays_o", "grad/rays_d"):
                r[k] = r[k][inv]
        for k, t in g_c.items():
            if t.grad is not None and float(t.grad.abs().max()) > 0:
                r["grad/" + k] = t.grad
        for k, t in p_c.items():
            if t.grad is not None and float(t.grad.abs().max()) > 0:
                r["grad/param/" + k] = t.grad
        refs[form] = un(r) if un is not None else r
    if (False, False, None) in refs:
        refs[False] = refs[(False, False, None)]
    if (True, False, None) in refs:
        refs[True] = refs[(True, False, None)]
    return refs


# --- C1 (BASELINE configs[0]) golden cases: tests/golden/make_golden_c1.py ---------------
C1_CASES = [
    # name, middle-grid scale, middle occupancy bias (None: the initialiser's), upstream seed
    ("c1_room0", 1.0, None, 71),
    ("c1_room0_spread", 30.0, -0.55, 72),
]


def c1_inputs(name):
    """(scene, grids, params, rays (ro, rd)) of a C1 golden case, regenerated from the seeds
    the generator used (init_grids seed 0 as bench.build_workload, build_default_nice seed
    0 = the reference's get_model under torch.manual_seed(0), synth_rays seed 1000)."""
    from nicecore import decoder as D
    from nicecore import scene as S
    scale, bias = next((s, b) for n, s, b, _ in C1_CASES if n == name)
    sc = S.make_scene("replica_room0")
    grids = S.init_grids(sc.shapes, generator=torch.Generator().manual_seed(0))
    grids = {k: (v * scale if k == "grid_middle" else v).contiguous() for k, v in grids.items()}
    m = D.build_default_nice(seed=0)
    if bias is not None:
        with torch.no_grad():
            m.middle_decoder.output_linear.bias.fill_(bias)
    params = {k: v.detach().clone() for k, v in m.named_parameters()}
    ro, rd, _, _ = S.synth_rays(sc, 200, seed=1000)
    return sc, grids, params, (ro, rd)


def c2_args(**over):
    """bench.py's default C2 arguments (Replica room0, 1000 rays, stage color, BA)."""
    import types
    a = dict(scene="replica_room0", rays=1000, stage="color", mode="ba", layout="channels_last",
             sparse_grads="auto", frustum="off", overlap="off", fix_fine=False, render_depth="target",
             param_grads="direct", eager=True, iteration=False)
    a.update(over)
    return types.SimpleNamespace(**a)


# --- a second float32 implementation: the same network with its units permuted ------------
# Reordering the rays only changes the reductions over points; every point's own arithmetic
# (each dot product's summation order) stays the oracle's.  Permuting the hidden units of
# every layer, the Fourier features and the grid channels gives a network that computes the
# same function with every dot product summed in another order -- another float32
# implementation, as the HIP path is one.  Gradients are mapped back to the original order.
_DECODER_GRID = {"coarse": "grid_coarse", "middle": "grid_middle", "fine": "grid_fine", "color": "grid_color"}


def permuted_problem(grids, params, seed):
    """(grids', params', unpermute): grids' channels and every decoder's units permuted;
    unpermute({name: grad'}) -> {name: grad} in the original order (grid and parameter
    gradients; other entries are returned unchanged)."""
    gen = torch.Generator().manual_seed(seed)
    rp = lambda n: torch.randperm(n, generator=gen)
    rho = {k: rp(v.shape[1]) for k, v in grids.items()}
    new_g = {k: v[:, rho[k]].contiguous() for k, v in grids.items()}
    idx = {}  # param name -> (row index | None, col index | None)
    decs = sorted({n.split(".")[0][:-len("_decoder")] for n in params})
    for d in decs:
        pre = d + "_decoder."
        xyz = d != "coarse"
        pi = [rp(32) for _ in range(5)]
        ident = torch.arange(32)  # a decoder whose grid is not in the problem (C5 windows: no coarse grid)
        if d == "fine":
            cin = torch.cat([rho.get("grid_fine", ident), 32 + rho.get("grid_middle", ident)])
        else:
            cin = rho.get(_DECODER_GRID[d], ident)
        sig = rp(93) if xyz else None
        for L in range(5):
            if L == 0:
                cols = sig if xyz else cin
            elif L == 3:
                cols = torch.cat([sig, 93 + pi[2]]) if xyz else torch.cat([cin, 32 + pi[2]])
            else:
                cols = pi[L - 1]
            idx[f"{pre}pts_linears.{L}.weight"] = (pi[L], cols)
            idx[f"{pre}pts_linears.{L}.bias"] = (pi[L], None)
            if xyz:
                idx[f"{pre}fc_c.{L}.weight"] = (pi[L], cin)
                idx[f"{pre}fc_c.{L}.bias"] = (pi[L], None)
        if xyz:
            idx[pre + "embedder._B"] = (None, sig)
        idx[pre + "output_linear.weight"] = (None, pi[4])

    def fwd(t, ri, ci):
        if ri is not None:
            t = t[ri]
        if ci is not None:
            t = t[:, ci]
        return t.contiguous()

    new_p = {n: fwd(v, *idx[n]) if n in idx else v for n, v in params.items()}

    def unpermute(out):
        res = dict(out)
        for k, v in out.items():
            if k.startswith("grad/param/") and k[len("grad/param/"):] in idx:
                ri, ci = idx[k[len("grad/param/"):]]
                g = torch.zeros_like(v)
                rows = ri if ri is not None else torch.arange(v.shape[0])
                if v.dim() == 1:
                    g[rows] = v
                else:
                    cols = ci if ci is not None else torch.arange(v.shape[1])
                    g[rows[:, None], cols[None, :]] = v
                res[k] = g
            elif k.startswith("grad/grid_") and k[len("grad/"):] in rho:
                g = torch.zeros_like(v)
                g[:, rho[k[len("grad/"):]]] = v
                res[k] = g
        return res
    return new_g, new_p, unpermute


def oracle_render_grads_permuted(grids, params, dec_b, bound, ro, rd, stage, gt, upstream, seed, depth_max=None):
    """oracle_render_grads (float32) of the unit-permuted network, in the original order."""
    g2, p2, un = permuted_problem(grids, params, seed)
    return un(oracle_render_grads(g2, p2, dec_b, bound, ro, rd, stage, gt, upstream, depth_max=depth_max))


def oracle_elementwise_gate(title, got, grids, params, dec_b, bound, ro, rd, stage, gt, upstream, depth_max=None):
    """The per-element gate (elementwise_vs_truth) of a HIP result ``got`` on any inputs:
    truth = the float64 oracle with the reference's float32 input roundings, refs = the
    float32 oracle and two unit-permuted float32 oracles; prints the table and returns the
    failing tensors, plus any gradient HIP produces that the reference does not (must be
    zero), under "extra"."""
    args = (grids, params, dec_b, bound, ro, rd, stage, gt, upstream)
    truth = oracle_render_grads(*args, f64=True, round_inputs=True, depth_max=depth_max)
    ref32 = oracle_render_grads(*args, depth_max=depth_max)
    refs = [ref32] + [oracle_render_grads_permuted(*args, seed=s, depth_max=depth_max) for s in (1, 2)]
    truth = {k: v for k, v in truth.items() if k in ref32}
    bad = report_elementwise(title, elementwise_vs_truth(got, refs, truth))
    extra = [k for k in got if k.startswith("grad/") and k not in ref32 and float(got[k].abs().max()) > 0]
    if extra:
        bad["extra"] = extra
    return bad
