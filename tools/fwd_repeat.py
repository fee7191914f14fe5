"""Forward determinism stress: render the same rays N times (render_img-sized chunks and
a C2 batch) and require bit-identical outputs (split-f16 forward).  GPU box.
    python tools/fwd_repeat.py [runs]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "nice-slam-annotation_amd")):
    sys.path.insert(0, p)
import torch  # noqa: E402
from nicecore import decoder as D  # noqa: E402
from nicecore import scene as S  # noqa: E402
from parity_common import build_model, make_renderer  # noqa: E402

runs = int(sys.argv[1]) if len(sys.argv) > 1 else 20
sc = S.make_scene("replica_room0")
grids = S.init_grids(sc.shapes, generator=torch.Generator().manual_seed(0), std={k: 0.3 for k in S.GRID_STD})
model = build_model(dict(D.build_default_nice(seed=0).state_dict()), sc.bound, sc.bound * 2, "cuda")
bad = 0
for cl in (False, True):
    g = {k: (v.cuda().contiguous(memory_format=torch.channels_last_3d) if cl else v.cuda()) for k, v in grids.items()}
    for n in (1000, 100000):
        ro, rd, dep, _ = S.synth_rays(sc, n, seed=7)
        ro, rd, dep = ro.cuda(), rd.cuda(), dep.cuda()
        r = make_renderer(sc.bound, H=sc.H, W=sc.W)
        ref = None
        with torch.no_grad():
            for k in range(runs):
                d, v, c = r.render_batch_ray(g, model, rd, ro, "cuda", "color", dep)
                out = torch.cat([d, v, c.double().reshape(-1)])
                if ref is None:
                    ref = out.clone()
                elif not torch.equal(out, ref):
                    bad += 1
                    print(f"cl={int(cl)} n={n} run {k}: differs, max {float((out - ref).abs().max()):.3e}", flush=True)
        print(f"cl={int(cl)} n={n}: {runs} runs done", flush=True)
print("bad runs:", bad)
sys.exit(1 if bad else 0)
