"""Repeat one golden case N times and print the rays-gradient errors of each run
(flakiness probe; GPU box).   python tools/parity_repeat.py <case> <channels_last> <N>"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "nice-slam-annotation_amd")):
    sys.path.insert(0, p)
import torch  # noqa: E402
from parity_common import compare, run_case  # noqa: E402

case, cl, n = sys.argv[1], bool(int(sys.argv[2])), int(sys.argv[3])
want = tuple(sys.argv[4].split(",")) if len(sys.argv) > 4 else ("rays", "grids", "params")
prev = None
prev_out = None
for k in range(n):
    rec, got = run_case(case, channels_last=cl, want=want)
    e = compare(rec, got)
    d = "" if prev is None else f" max|Δ rays_o| vs previous run {float((got['grad/rays_o'] - prev).abs().max()):.3e}"
    prev = got["grad/rays_o"]
    outs = torch.cat([got["depth"].reshape(-1), got["color"].double().reshape(-1)])
    if prev_out is not None and not torch.equal(outs, prev_out):
        print("   forward outputs differ from the previous run by", float((outs - prev_out).abs().max()), flush=True)
    prev_out = outs
    print(f"run {k}: rays_o {e['grad/rays_o']:.2e} rays_d {e['grad/rays_d']:.2e} grid_fine {e.get('grad/grid_fine', 0):.2e} depth {e['depth']:.2e}{d}",
          flush=True)
    if e["grad/rays_o"] > 1e-4:
        bad = (got["grad/rays_o"] - rec["grad/rays_o"]).abs().sum(1)
        idx = torch.nonzero(bad > 1e-4 * rec["grad/rays_o"].abs().max()).flatten().tolist()
        print("   bad rays:", idx[:20], flush=True)
