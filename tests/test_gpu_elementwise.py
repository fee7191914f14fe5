"""Per-element parity against a float64 truth.

Every other parity test scores a tensor by its largest error over its largest value
(parity_common.rel_err).  That metric hides a wrong gradient on a lightly-touched voxel
or a low-weight ray while it stays below the gate's fraction of the tensor's maximum.
Here every element of every output and gradient is held to (parity_common.ELEM_FACTOR)

    |hip - t| <= 4 max_k |ref_k - t| + 4 rms(ref_0 - t)

t: the oracle in float64 keeping the reference's float32 input roundings (p.float(), the
float32 lookup coordinates) -- the exact value of the reference's float32 program;
ref_0: the reference's own vectors (tests/golden, produced by importing /root/reference)
for the golden and init-std cases, the float32 oracle for the C2 benchmark workload;
ref_1, ref_2: the float32 oracle on the network with its hidden units, Fourier features and
grid channels permuted (parity_common.permuted_problem: the same function, every dot
product summed in another order -- independent float32 roundings at every point, as another
implementation has; reordering the rays alone would leave every point's arithmetic the
oracle's).  Checked on the CPU: the reference's own vectors against three such permutations,
and each permutation against the other references, stay below 0.8 of this gate.  The floor, 4x the reference's own RMS error over the tensor, is far
below the tensor's max (a voxel's wrong gradient shows unless it is within float32 noise).
Grid gradients must also have ref_0's support: the same voxels with a non-zero gradient
(a dropped or mis-addressed scatter of any size shows there).  The C2 workload is scored
both eager and as the graph-replayed step bench.py times (bench.make_step(...)[1]).
Each test prints the per-tensor table: worst per-element ratio, relative L2 and
max-normalised errors of HIP and of ref_0, and the floor.

Why not a fixed atol of 1e-6 of the max (VERDICT r04's suggestion): the reference's own
float32 error is above it -- up to 5.6e-6 of the max on the golden decoder gradients
(profiles/r05/elementwise/), so an independent float32 implementation cannot meet it; and
with a single float32 reference, an element where it happens to land on the truth
leaves no room for any other summation order.

Reference: src/utils/Renderer.py:95-262 (render_batch_ray), src/conv_onet/models/
decoder.py:179-219 (grid_sample + MLP; the grid_sampler_3d backward scatter at :186),
src/Mapper.py:603-612 (the Mapper loss)."""
import pytest
import torch

from conftest import CASE_NAMES, INITSTD_CASES, load_case
from parity_common import (C1_CASES, c1_inputs, c2_args, case_stage, hip_render_grads, collect_step, oracle_mapper_refs, oracle_render_grads,
                           oracle_render_grads_permuted, report_elementwise, elementwise_vs_truth, run_case,
                           scene_of)
from conftest import load_scene


# Every golden case passes strict (round 6).  fine_depth (20 rays, the fine stage) failed
# through round 5 at 1.14 of the gate on 1-2 elements of the fine decoder's deeper weight
# gradients; the cause was the forward's Fourier features: the hardware v_sin_f32 after a
# [-pi, pi] reduction had 3.8e-7 absolute error (5 float32 ulps of a feature) where the
# reference's sinf is within an ulp.  Fed the truth's d raw, the HIP decoder backward alone
# sits at float32 level (tools/diag_chain.py); d raw's error is the forward's occupancy
# error (the compositing adds 2e-7), and the sin error was the forward's one HIP-specific
# part of it.  nc_device.h fourier_sin is now a Cody-Waite + minimax form at 6.9e-8
# (profiles/r06/numerics/).
_GOLDEN = CASE_NAMES + INITSTD_CASES


@pytest.mark.gpu
@pytest.mark.parametrize("case", _GOLDEN)
@pytest.mark.parametrize("channels_last", [False, True])
def test_golden_elementwise(case, channels_last):
    rec, got = run_case(case, channels_last=channels_last)
    bound, cbound, grids, params = load_scene(scene_of(case))
    stage, with_depth = case_stage(case)
    dec_b = {"coarse": cbound, "middle": bound, "fine": bound, "color": bound}
    gt = rec["gt_depth"] if with_depth else None
    args = (grids, params, dec_b, bound, rec["rays_o"], rec["rays_d"], stage, gt,
            (rec["g_depth"], rec["g_var"], rec["g_color"]))
    truth = oracle_render_grads(*args, f64=True, round_inputs=True)
    truth = {k: v for k, v in truth.items() if k in rec}  # the tensors the reference produced
    p1 = oracle_render_grads_permuted(*args, seed=1)
    p2 = oracle_render_grads_permuted(*args, seed=2)
    res = elementwise_vs_truth(got, [rec, p1, p2], truth)
    _dump(f"golden_{case}_{int(channels_last)}", got, [rec, p1, p2], truth)
    bad = report_elementwise(f"{case} {'channels_last' if channels_last else 'ncdhw'}", res)
    assert not bad, bad


@pytest.mark.gpu
@pytest.mark.parametrize("case", [c[0] for c in C1_CASES])
@pytest.mark.parametrize("channels_last", [False, True])
def test_c1_golden_elementwise(case, channels_last):
    """BASELINE configs[0] (C1: Replica room0, 200 rays x 32 samples, stage middle) against
    the reference's own vectors at that size (tests/golden/make_golden_c1.py), per element,
    with the grid-support check on grid_middle."""
    sc, grids, params, (ro, rd) = c1_inputs(case)
    rec = load_case(case)
    up = (rec["g_depth"], rec["g_var"], rec["g_color"])
    dec_b = {"coarse": sc.bound * 2, "middle": sc.bound, "fine": sc.bound, "color": sc.bound}
    got = hip_render_grads(grids, params, sc.bound, sc.bound * 2, ro, rd, "middle", None, up,
                           channels_last=channels_last)
    args = (grids, params, dec_b, sc.bound, ro, rd, "middle", None, up)
    truth = oracle_render_grads(*args, f64=True, round_inputs=True)
    truth = {k: v for k, v in truth.items() if k in rec}
    p1 = oracle_render_grads_permuted(*args, seed=1)
    p2 = oracle_render_grads_permuted(*args, seed=2)
    res = elementwise_vs_truth(got, [rec, p1, p2], truth)
    bad = report_elementwise(f"{case} {'channels_last' if channels_last else 'ncdhw'}", res)
    extra = [k for k in got if k.startswith("grad/") and k not in rec and float(got[k].abs().max()) > 0]
    assert not extra, extra  # a gradient the reference does not produce must be zero
    assert not bad, bad


def _dump(name, got, refs, truth):
    """NICECORE_ELEM_DUMP=<dir>: save the compared tensors (for offline study of the gate)."""
    import os
    d = os.environ.get("NICECORE_ELEM_DUMP")
    if d:
        os.makedirs(d, exist_ok=True)
        torch.save({"got": got, "refs": refs, "truth": truth}, os.path.join(d, name + ".pt"))


def _c2_eager_and_graphed():
    import bench
    dev = torch.device("cuda", 0)
    args = c2_args(eager=False)
    w = bench.build_workload(args, 0, dev)
    eager, graphed = bench.make_step(w, args, 1, dev)
    out = {}
    for _ in range(3):  # several replays: each rewrites every gradient from zero
        graphed()
    torch.cuda.synchronize()
    out["graphed"] = collect_step(w["grids"], w["model"], w["ro"], w["rd"], None, graphed.step.out)
    # eager, with the outputs: the call the captured body makes (bench.make_step.body)
    grids, model = w["grids"], w["model"]
    for t in list(grids.values()) + list(model.parameters()) + [w["ro"], w["rd"]]:
        t.grad = None
    d, u, c, loss = w["renderer"].render_batch_loss(grids, model, w["rd"], w["ro"], dev, "color", w["gt"],
                                                    w["gtc"], **bench.LOSS_KW["ba"]("color"),
                                                    render_gt_depth="target")
    loss.backward()
    torch.cuda.synchronize()
    out["eager"] = collect_step(grids, model, w["ro"], w["rd"], (d, u, c), loss)
    return w, out


@pytest.mark.gpu
def test_c2_workload_elementwise_eager_and_graphed():
    """bench.py's C2 workload (room0, 1000 rays x 48 samples, the reference's grid_init
    statistics, channels-last grids, the fused Mapper loss, BA gradients): the eager step and
    the graph-replayed step the bench times, each against the oracle's float32 / float64
    render + loss + backward, per element; and the two HIP forms against each other."""
    import bench
    w, out = _c2_eager_and_graphed()
    f32, f32r, f32p, t64 = (False, False, None), (False, False, None, 1), (False, False, None, 2), (True, True, None)
    refs = oracle_mapper_refs(w, bench.LOSS_KW["ba"]("color"), forms=(f32, f32r, f32p, t64))
    bad = {}
    for form in ("eager", "graphed"):
        truth = refs[t64] if form == "eager" else {k: v for k, v in refs[t64].items()
                                                   if k not in ("depth", "var", "color")}
        res = elementwise_vs_truth(out[form], [refs[f32], refs[f32r], refs[f32p]], truth)
        bad.update({f"{form}:{k}": v for k, v in report_elementwise(f"C2 {form}", res).items()})
    # the replayed step against the eager one: ray and parameter gradients bit-identical
    # (fixed-order reductions), grid gradients to float-atomic order
    for k, g in out["graphed"].items():
        v = out["eager"][k]
        if k.startswith("grad/grid_"):
            assert float((g - v).abs().max()) <= 1e-6 * float(v.abs().max()), k
        else:
            assert torch.equal(g, v), k
    assert not bad, bad
