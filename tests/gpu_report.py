"""Print the scale-aware error of every output / gradient of every golden case on
the HIP core (diagnostic companion of test_gpu_parity.py; run on the GPU box)."""
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import conftest  # noqa: E402,F401  (import paths)
from conftest import CASE_NAMES  # noqa: E402
from parity_common import compare, run_case  # noqa: E402

def room0_report(n_rays, stage="color"):
    """Room0-geometry case: forward with / without NC_SAVE_FOR_BACKWARD and all
    gradients, each vs the float64 oracle (err_hip, err_fp32_oracle, allowed)."""
    import torch
    from parity_common import make_renderer, build_model, oracle_render_grads, score_vs_truth
    from test_gpu_parity import _room0_case
    sc, grids, params, ro, rd, dep = _room0_case(n_rays, stage)
    cb = sc.bound * 2
    dec_b = {"coarse": cb, "middle": sc.bound, "fine": sc.bound, "color": sc.bound}
    gt = dep if stage in ("color", "fine") else None
    gen = torch.Generator().manual_seed(11)
    up = (torch.randn(n_rays, generator=gen, dtype=torch.float64),
          torch.randn(n_rays, generator=gen, dtype=torch.float64), torch.randn(n_rays, 3, generator=gen))
    ref32 = oracle_render_grads(grids, params, dec_b, sc.bound, ro, rd, stage, gt, up)
    ref64 = oracle_render_grads(grids, params, dec_b, sc.bound, ro, rd, stage, gt, up, f64=True)
    model = build_model(params, sc.bound, cb, "cuda")
    r = make_renderer(sc.bound)
    g_g = {k: v.cuda().contiguous(memory_format=torch.channels_last_3d) for k, v in grids.items()}
    gtc = gt.cuda() if gt is not None else None
    with torch.no_grad():
        d0, v0, c0 = r.render_batch_ray(g_g, model, rd.cuda(), ro.cuda(), "cuda", stage, gtc)
    ro_g, rd_g = ro.cuda().requires_grad_(True), rd.cuda().requires_grad_(True)
    for v in g_g.values():
        v.requires_grad_(True)
    d_g, v_g, c_g = r.render_batch_ray(g_g, model, rd_g, ro_g, "cuda", stage, gtc)
    print(f"== room0 {stage} N={n_rays}: no-save vs save forward max|diff| "
          f"depth {float((d0 - d_g).abs().max()):.3e} color {float((c0 - c_g).abs().max()):.3e}")
    torch.autograd.backward([d_g, v_g, c_g], [t.cuda() for t in up])
    got = {"depth": d_g.detach().cpu(), "var": v_g.detach().cpu(), "color": c_g.detach().cpu(),
           "grad/rays_o": ro_g.grad.cpu(), "grad/rays_d": rd_g.grad.cpu(),
           "nosave/depth": d0.cpu(), "nosave/color": c0.cpu()}
    for k, v in g_g.items():
        if v.grad is not None:
            got["grad/" + k] = v.grad.cpu()
    for n, p in model.named_parameters():
        if p.grad is not None:
            got["grad/param/" + n] = p.grad.cpu()
    ref64 = dict(ref64, **{"nosave/depth": ref64["depth"], "nosave/color": ref64["color"]})
    ref32 = dict(ref32, **{"nosave/depth": ref32["depth"], "nosave/color": ref32["color"]})
    worst = 0.0
    for k, (e, e32, allowed) in sorted(score_vs_truth(got, ref32, ref64).items(), key=lambda kv: -kv[1][0]):
        print(f"   {e:10.3e} (fp32 oracle {e32:9.2e}, allowed {allowed:9.2e}) {'FAIL' if e > allowed else ''} {k}")
        worst = max(worst, e / allowed)
    print("WORST/allowed", worst)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--room0":
        for n in sys.argv[2:] or ["256"]:
            room0_report(int(n))
        sys.exit(0)
    worst = 0.0
    for cl in (False, True):
        for case in CASE_NAMES:
            try:
                rec, got = run_case(case, channels_last=cl)
            except Exception:
                print(f"== {case} channels_last={cl}: EXCEPTION")
                traceback.print_exc()
                continue
            errs = compare(rec, got)
            missing = [k for k in rec if k.startswith("grad/") and k not in got]
            print(f"== {case} channels_last={cl} missing={missing}")
            for k, e in sorted(errs.items(), key=lambda kv: -kv[1]):
                flag = "" if k in rec else "  (ref has no grad: abs max)"
                print(f"   {e:10.3e}  {k}{flag}")
                worst = max(worst, e)
    print("WORST", worst)
