"""Run the same render + mapper loss + backward twice and diff the render workspaces
(debug tool: which buffer of k_mlp_dx's outputs differs between identical runs).
    python tools/ws_diff.py [rays] [runs]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "nice-slam-annotation_amd")):
    sys.path.insert(0, p)
import torch  # noqa: E402
from nicecore import render_fn as RF  # noqa: E402
from nicecore import scene as S  # noqa: E402
from parity_common import build_model, make_renderer  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
runs = int(sys.argv[2]) if len(sys.argv) > 2 else 8
cl = len(sys.argv) > 3 and sys.argv[3] == "cl"
kept = []
orig = RF.NiceRenderFn.backward


def hooked(ctx, *a):
    out = orig(ctx, *a)
    kept.append(ctx.ws.detach().clone())  # same stream: ordered after the backward's kernels
    return out


RF.NiceRenderFn.backward = staticmethod(hooked)
sc = S.make_scene("replica_room0")
grids = S.init_grids(sc.shapes, generator=torch.Generator().manual_seed(0))
from nicecore import decoder as D  # noqa: E402
params = dict(D.build_default_nice(seed=0).state_dict())
model = build_model(params, sc.bound, sc.bound * 2, "cuda")
g = {k: (v.cuda().contiguous(memory_format=torch.channels_last_3d) if cl else v.cuda()).requires_grad_(True)
     for k, v in grids.items()}
ro, rd, dep, col = S.synth_rays(sc, N, seed=3)
r = make_renderer(sc.bound)
P = N * 48
nj = 3
ref_grads = None
for k in range(runs):
    ro_ = ro.cuda().requires_grad_(True)
    rd_ = rd.cuda().requires_grad_(True)
    d, v, c, L = r.render_batch_loss(g, model, rd_, ro_, "cuda", "color", dep.cuda(), col.cuda(), loss="mapper",
                                     w_color_loss=0.2, color_term=True)
    L.backward()
    gr = torch.cat([ro_.grad.reshape(-1), rd_.grad.reshape(-1)]).double().cpu()
    if ref_grads is None:
        ref_grads = gr
    else:
        print(f"run {k}: max |d rays grad| vs run 0: {float((gr - ref_grads).abs().max()):.3e}", flush=True)
    for t in list(g.values()) + list(model.parameters()):
        t.grad = None
ws0 = kept[0]
# workspace layout (nc_abi.hip layout(): 256-B aligned takes)
off = 0
names = []


def take(name, nbytes):
    global off
    names.append((name, off, nbytes))
    off = (off + nbytes + 255) // 256 * 256


take("dmax", 16); take("z", P * 8); take("pts", P * 24); take("xyz", nj * P * 16); take("pf", P * 16)
take("occ", nj * P * 4); take("rgb", P * 12); take("gocc", P * 4); take("grgb", P * 12); take("dpts", nj * P * 24)
take("coef_d", N * 8); take("coef_c", N * 12)
for k, ws in enumerate(kept[1:], 1):
    diff = (ws != ws0)
    if not bool(diff.any()):
        print(f"run {k}: workspace identical")
        continue
    idx = torch.nonzero(diff).flatten()
    msg = []
    for name, o, n in names:
        m = ((idx >= o) & (idx < o + n))
        if bool(m.any()):
            first = int(idx[m][0]) - o
            msg.append(f"{name} ({int(m.sum())} bytes, first at +{first})")
    rest = int(((idx >= off)).sum())
    print(f"run {k}: differing: " + ", ".join(msg) + f"; beyond the per-point buffers (records, slabs): {rest} bytes")
    dp = [x for x in names if x[0] == "dpts"][0]
    a = ws0[dp[1]:dp[1] + dp[2]].view(torch.float64).reshape(nj, P, 3)
    b = ws[dp[1]:dp[1] + dp[2]].view(torch.float64).reshape(nj, P, 3)
    dd = (a - b).abs().amax(2)
    if bool((dd > 0).any()):
        j, p = [int(x) for x in torch.nonzero(dd > 0)[0]]
        print(f"   dpts first diff: job {j} point {p} (ray {p // 48}, sample {p % 48}, tile {p // 16}, lane i {p % 16}): "
              f"{a[j, p].tolist()} vs {b[j, p].tolist()}; {int((dd > 0).sum())} points differ")
