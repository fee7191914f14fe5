"""Benchmark: rendered rays/s (fwd+bwd) of NICE-SLAM's render_batch_ray hot path.

Workload (BASELINE.json configs[1]): Replica room0 scene (snapped bound, grid
shapes middle [21,28,37], fine/color [43,56,74]), 1000 rays x 48 samples per GPU
(32 stratified + 16 surface), stage 'color' (middle + fine + color decoders),
mapper/BA gradients (rays, the three grids and every decoder parameter), the
mapper's L1 loss (src/Mapper.py:603-612) and backward.  Synthetic seeded rays and
random-init decoders / N(0,.) grids (no datasets or checkpoints exist here).

One step = render_batch_ray + loss + backward (+ for N>1 the RCCL all-reduce of
grid and decoder gradients, and the all-reduce(MAX) of the batch-global depth
bound that render_batch_ray needs before sampling).  Weak scaling: every rank
renders its own 1000 rays.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--mode ba|tracker]

--gpus N > 1 either runs under torch.distributed.run (WORLD_SIZE set: one rank of N) or,
without a launcher, starts the N ranks itself (launch_ranks: torch.multiprocessing spawn,
MASTER_ADDR 127.0.0.1, a free port).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
import types

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "nice-slam-annotation_amd")
for _p in (REPO, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402

METRIC = "rendered rays/sec (fwd+bwd), Replica room0 1000 rays×48 samples, 1/2/4/8 GPU"
FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: f32 MFMA dense peak (= f32 vector peak)
F16_MFMA_PEAK_TFLOPS = 2500.0   # MI355X_MICROARCH.md: dense f16/bf16 MFMA peak
# k_mlp_fwd runs every decoder GEMM as three f16 MFMAs (hi*hi + hi*lo + lo*hi, f32
# accumulate; csrc/nc_device.h), so its matrix peak in algorithmic f32 FLOP/s is a third of
# the f16 peak; k_mlp_dx and k_mlp_dw run the exact-f32 MFMA
SPLIT16_PEAK_TFLOPS = F16_MFMA_PEAK_TFLOPS / 3
MFMA_PEAK = {"k_mlp_fwd": SPLIT16_PEAK_TFLOPS, "k_mlp_dx": FP32_MFMA_PEAK_TFLOPS, "k_mlp_dw": FP32_MFMA_PEAK_TFLOPS,
             "k_grid_gather": FP32_MFMA_PEAK_TFLOPS}
HBM_PEAK_GBS = 8000.0
# MI355X_MICROARCH.md "Global float atomics": no-return f32 atomics execute at the memory side,
# chip-wide ~1.3 TB/s of added bytes (1.26-1.36) whatever the contention pattern
ATOMIC_PEAK_GBS = 1300.0
MAC = {"coarse": 6176, "middle": 15479, "fine": 20599, "color": 15575}  # per point
TRI_FLOP = 8 * 32 * 2  # one trilinear lookup of 32 channels
# dX-chain MACs per point: the fine decoder's fc_c input gradient is only taken for its
# own 32 grid channels (the middle features enter under no_grad, decoder.py:196-202)
MAC_DX = {"coarse": 6176, "middle": 15479, "fine": 20599 - 5 * 32 * 32, "color": 15575}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--rays", type=int, default=1000)
    ap.add_argument("--scene", default="replica_room0")
    ap.add_argument("--stage", default="color")
    ap.add_argument("--mode", default="ba", choices=["ba", "tracker"])
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="bounded CPU-oracle sample (0 disables)")
    ap.add_argument("--layout", default="channels_last", choices=["channels_last", "ncdhw"])
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend for N>1 (nccl = RCCL; gloo only to rehearse "
                         "the multi-rank path on one GPU)")
    ap.add_argument("--sparse-grads", default="auto", choices=["auto", "on", "off"],
                    help="grid gradients as touched-voxel rows (nicecore.sparse); auto = on for "
                         "grids too large for a dense gradient per iteration (C5)")
    ap.add_argument("--overlap", default="auto", choices=["auto", "on", "off"],
                    help="split the backward (render_fn.DeferParamGrads) so the grid-gradient "
                         "all-reduce overlaps the decoder weight gradients; auto = on for N > 1 "
                         "(BA mode, dense grid gradients)")
    ap.add_argument("--frustum", default="auto", choices=["auto", "on", "off"],
                    help="N > 1 grid-gradient exchange over the voxels of the current frame's frustum "
                         "only (the Mapper's frustum_feature_selection, configs/nice_slam.yaml:74, "
                         "Mapper.py:371-414: the other voxels are not optimised); auto = on for N > 1 "
                         "(BA mode, dense channels-last grid gradients)")
    ap.add_argument("--iteration", action="store_true",
                    help="also time the whole Mapper iteration with the Adam step (nicecore.optim.Adam, "
                         "capturable) in the same hipGraph; reported as mapper_iteration_ms")
    ap.add_argument("--fix-fine", action="store_true",
                    help="the Mapper's fix_fine=True (configs/nice_slam.yaml:62, Mapper.py:416-424): only "
                         "the color decoder's parameters require grad, the ones the Mapper optimises. "
                         "Default: every decoder parameter requires grad, as in the reference, whose "
                         "autograd computes (and never uses) the middle and fine decoder gradients")
    ap.add_argument("--render-depth", default="target", choices=["target", "none"],
                    help="render with the loss target as gt_depth (Mapper / Tracker, S = 48) or "
                         "without one (S = 32: BASELINE configs[0], the reference's CPU plumbing "
                         "case C1; the loss still compares with the targets)")
    ap.add_argument("--param-grads", default="direct", choices=["autograd", "direct"],
                    help="how the decoder parameters get .grad in the drop-in step (render_fn.param_inputs): "
                         "written by the backward itself (the library default) or through autograd's "
                         "AccumulateGrad (rendering.param_grads: autograd); both eager times are reported")
    ap.add_argument("--eager", action="store_true",
                    help="time the eager step instead of its hipGraph replay "
                         "(nicecore.graph.GraphedStep)")
    ap.add_argument("--global-batch", action="store_true",
                    help="draw ONE batch of N x --rays rays (seed 1000) and give rank r its contiguous shard "
                         "(distributed.shard), instead of --rays fresh rays per rank: the N-rank step then "
                         "computes the gradients of the 1-rank step over the whole batch (tests)")
    ap.add_argument("--global-rays", type=int, default=0,
                    help="one batch of this many rays in total (seed 1000), rank r rendering its contiguous "
                         "shard (distributed.shard_bounds: the first total %% N ranks get one ray more); "
                         "--rays is then the shard size (tests: uneven shards)")
    ap.add_argument("--dump-grads", default=None,
                    help="after the timed steps run one more step and have rank 0 save its exchanged "
                         "gradients (decoder parameters; grid rows of the frustum, or whole grids without "
                         "one) with torch.save to this path (tests/test_gpu_bench_ranks.py)")
    return ap.parse_args()


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spawned_rank(local, world, port, argv):
    """Entry of one rank started by launch_ranks (a fresh interpreter: torch.multiprocessing
    'spawn'), with the environment torch.distributed.run would have given it."""
    os.environ.update(RANK=str(local), LOCAL_RANK=str(local), WORLD_SIZE=str(world),
                      LOCAL_WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    sys.argv = argv
    main()


def launch_ranks(args) -> None:
    """``python bench.py --gpus N`` without an external launcher: start N rank processes
    (one per GPU) and wait for them.  The parent makes no HIP call (device_count() does
    not initialise the runtime on this image), so no rank inherits a GPU context."""
    import torch.multiprocessing as mp
    n = args.gpus
    have = torch.cuda.device_count()
    if args.backend == "nccl" and n > have:
        raise SystemExit(f"bench.py: --gpus {n} but only {have} HIP device(s) are visible "
                         f"(RCCL needs one GPU per rank; --backend gloo rehearses N ranks on fewer GPUs)")
    if have == 0:
        raise SystemExit("bench.py: no HIP device visible")
    mp.spawn(_spawned_rank, args=(n, _free_port(), list(sys.argv)), nprocs=n, join=True)


def setup_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} ranks were launched")
    if world > 1:
        import torch.distributed as dist
        dev = local % torch.cuda.device_count()  # == local on a node with >= N GPUs
        torch.cuda.set_device(dev)
        if args.backend == "nccl":  # RCCL
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:  # rehearsal of the N>1 path with several ranks on one GPU
            dist.init_process_group(args.backend)
        if dist.get_world_size() != args.gpus:
            raise SystemExit(f"bench.py: process group has {dist.get_world_size()} ranks, --gpus {args.gpus}")
    else:
        torch.cuda.set_device(0)
    return world, rank, local


def frustum_rows(sc, grids, device):
    """Voxel rows of each optimised grid inside the current frame's frustum
    (nicecore.frustum, Mapper.get_mask_from_c2w): the camera is the first synthetic pose
    of rank 0's seed on every rank, so all ranks exchange the same rows; the depth image
    is the bound's diagonal everywhere (no surface in front of the walls), so the depth
    test keeps the whole frustum inside the bound."""
    from nicecore import scene as S
    from nicecore.frustum import FrustumSelector
    poses = []
    S.synth_rays(sc, 1, seed=1000, poses_out=poses)
    R, t = poses[0]
    c2w = torch.eye(4)
    c2w[:3, :3], c2w[:3, 3] = R, t
    depth = torch.full((sc.H, sc.W), float((sc.bound[:, 1] - sc.bound[:, 0]).norm()))
    sel = FrustumSelector(sc.bound, sc.H, sc.W, sc.fx, sc.fy, sc.cx, sc.cy, device)
    rows = {}
    for k, g in grids.items():
        if k == "grid_coarse" or not g.requires_grad:
            continue
        m = sel.grid_mask(c2w, k, g.shape[2:], depth)  # [Z, Y, X]
        rows[k] = m.reshape(-1).nonzero().squeeze(1)
    return rows


def build_workload(args, rank, device, world=1):
    from nicecore import decoder as D
    from nicecore import scene as S
    from nicecore.renderer import Renderer
    sc = S.make_scene(args.scene)
    if S.grids_bytes(sc.shapes) > (2 << 30):  # C5-sized grids: generated in HBM, no host copy
        grids = S.init_grids_device(sc.shapes, seed=rank, device=device,
                                    channels_last=(args.layout == "channels_last"))
    else:
        gen = torch.Generator().manual_seed(0)
        grids = S.init_grids(sc.shapes, generator=gen, device=device,
                             channels_last=(args.layout == "channels_last"))
    model = D.build_default_nice(seed=0).to(device)
    model.bound = sc.bound.to(device)
    for n in ("middle", "fine", "color"):
        getattr(model, n + "_decoder").bound = model.bound
    model.coarse_decoder.bound = (sc.bound * 2).to(device)
    if getattr(args, "global_rays", 0):  # one batch of a given total, possibly uneven shards
        from nicecore.distributed import shard
        ro, rd, dep, col = shard(rank, world, *S.synth_rays(sc, args.global_rays, seed=1000))
        args.rays = int(ro.shape[0])
    elif getattr(args, "global_batch", False):  # one batch over all ranks, contiguous shards
        from nicecore.distributed import shard
        ro, rd, dep, col = shard(rank, world, *S.synth_rays(sc, args.rays * world, seed=1000))
    else:
        ro, rd, dep, col = S.synth_rays(sc, args.rays, seed=1000 + rank)
    slam = types.SimpleNamespace(nice=True, bound=sc.bound, H=sc.H, W=sc.W, fx=sc.fx, fy=sc.fy,
                                 cx=sc.cx, cy=sc.cy)
    cfg = {"rendering": dict(S.DEFAULT_RENDERING, param_grads=getattr(args, "param_grads", "direct")), "scale": 1, "occupancy": True}
    renderer = Renderer(cfg, None, slam)
    ba = args.mode == "ba"
    for g in grids.values():
        g.requires_grad_(ba)
    for p in model.parameters():
        p.requires_grad_(ba)
    if args.fix_fine:  # only the color decoder is in the Mapper's optimizer
        for n in ("coarse", "middle", "fine"):
            for p in getattr(model, n + "_decoder").parameters():
                p.requires_grad_(False)
    sparse = None
    if ba and (args.sparse_grads == "on" or
               (args.sparse_grads == "auto" and S.grids_bytes(sc.shapes) > (2 << 30))):
        from nicecore.sparse import SparseGridGrads
        # rows for every corner of every lookup of one step: no growth after the first step
        sparse = SparseGridGrads(grids, capacity=8 * args.rays * 48)
    frustum = None
    if (ba and sparse is None and args.layout == "channels_last" and
            (args.frustum == "on" or (args.frustum == "auto" and world > 1))):
        frustum = frustum_rows(sc, grids, device)
        if world > 1:  # every rank must exchange the same rows (else the collective would hang)
            import torch.distributed as dist
            mine = torch.tensor([int(v.numel()) for v in frustum.values()] + [int(v.sum()) for v in frustum.values()],
                                dtype=torch.int64, device=device)
            lo, hi = mine.clone(), mine.clone()
            dist.all_reduce(lo, op=dist.ReduceOp.MIN)
            dist.all_reduce(hi, op=dist.ReduceOp.MAX)
            if not torch.equal(lo, hi):
                raise RuntimeError("frustum rows differ across ranks")
    w = dict(sc=sc, grids=grids, model=model, renderer=renderer,
             ro=ro.to(device).requires_grad_(True), rd=rd.to(device).requires_grad_(True),
             gt=dep.to(device), gtc=col.to(device), ba=ba, sparse=sparse, frustum=frustum)
    return w


# the callers' loss configuration (configs/nice_slam.yaml: mapping.w_color_loss 0.2,
# tracking.w_color_loss 0.5, use_color_in_tracking, handle_dynamic)
LOSS_KW = {
    "ba": lambda stage: dict(loss="mapper", w_color_loss=0.2, color_term=stage == "color"),
    "tracker": lambda stage: dict(loss="tracker", w_color_loss=0.5, color_term=True, handle_dynamic=True),
}


def make_step(w, args, world, device):
    """One iteration = [all-reduce(MAX) of the depth bound] -> render_batch_ray with the
    fused Mapper (BA) / Tracker loss -> backward -> [all-reduce of the gradients].  Returns the eager
    step and the graph-replayed step (render + loss + backward captured once into a
    hipGraph, nicecore.graph.GraphedStep; the collectives stay outside the graph)."""
    import torch.distributed as dist
    from nicecore import distributed as ND
    grids, model, renderer = w["grids"], w["model"], w["renderer"]
    ro, rd, gt, gtc = w["ro"], w["rd"], w["gt"], w["gtc"]
    params = [p for p in model.parameters() if p.requires_grad]
    sparse = w["sparse"]
    gvals = [g for k, g in grids.items() if g.requires_grad and (sparse is None or k not in sparse.rows)]
    dmax = gt.max().reshape(1).clone() if world > 1 else None  # static buffer
    one = torch.ones((), dtype=torch.float64, device=device)  # d loss / d loss, allocated once
    loss_kw = LOSS_KW[args.mode](args.stage)

    overlap = (w["ba"] and sparse is None and
               (args.overlap == "on" or (args.overlap == "auto" and world > 1)))
    from nicecore.render_fn import DeferParamGrads
    defer = DeferParamGrads() if overlap else None

    def pre():
        if world > 1:  # Renderer.py:157/:194 use max(gt_depth) over the whole (sharded) batch
            torch.amax(gt, dim=0, keepdim=True, out=dmax)
            dist.all_reduce(dmax, op=dist.ReduceOp.MAX)

    def body():
        for t in params + gvals + [ro, rd]:
            t.grad = None
        if sparse is not None:  # touched-voxel grid gradients: forget last step's rows
            sparse.zero_grad()
        if defer is not None:
            defer.clear()
        # render_batch_ray + the caller's loss in the same launches (k_loss):
        # Mapper.py:603-612 (BA mode) / Tracker.py:117-131 (tracker mode)
        depth, unc, color, loss = renderer.render_batch_loss(
            grids, model, rd, ro, device, args.stage, gt, gtc, **loss_kw, depth_max=dmax,
            sparse_grads=sparse, defer_param_grads=defer,
            render_gt_depth="target" if args.render_depth == "target" else None)
        loss.backward(one)  # = loss.backward(), without a fill kernel per step
        return loss

    frustum = w["frustum"]
    gkeys = [k for k, g in grids.items() if g.requires_grad and (sparse is None or k not in sparse.rows)]

    def grid_exchange_async():
        if frustum is None:  # one RCCL SUM over the core's shared gradient buffer
            return ND.allreduce_grads_async(gvals)
        # the frustum's voxel rows only (Mapper frustum feature selection): one RCCL SUM
        return ND.allreduce_rows_async([(grids[k].grad, frustum[k]) for k in gkeys
                                        if k in frustum and grids[k].grad is not None])

    def post():
        if world > 1 and w["ba"]:
            grid_exchange_async()()
            ND.allreduce_grads(params)
            if sparse is not None:  # union of the ranks' touched voxels, then one SUM per grid
                sparse.allreduce()

    def tail():  # the decoder weight gradients the split backward left out
        defer.run()

    def split_post(run_tail):
        # grid gradients are final: start their all-reduce, compute the weight
        # gradients meanwhile, then reduce those (small) once they exist
        finish = grid_exchange_async() if world > 1 else (lambda: None)
        run_tail()
        finish()
        if world > 1:
            ND.allreduce_grads(params)

    def eager():
        pre()
        body()
        if defer is None:
            post()
        else:
            split_post(tail)

    make_step.last_body = body
    graphed = None
    if not args.eager:
        from nicecore.graph import GraphedStep
        pre()
        g = GraphedStep(body)
        if defer is None:
            def graphed():
                pre()
                g()
                post()
        else:  # two captures: render + loss + backward without dW, then dW + reduction
            g2 = GraphedStep(tail)

            def graphed():
                pre()
                g()
                split_post(g2)
        graphed.step = g  # its .out: the loss of the last replay (tests score the replayed step)
    return eager, graphed


STAGE_DECODERS = {"coarse": ["coarse"], "middle": ["middle"], "fine": ["fine", "middle"],
                  "color": ["fine", "middle", "color"]}
# distinct trilinear lookups per point (k_grid_gather reads grid_middle once for the fine
# and middle decoders, MlpCtx::share_mid); lk_fwd of them are written out
LOOKUPS_UNIQUE = {"coarse": 1, "middle": 1, "fine": 2, "color": 3}
LOOKUPS_FWD = {"coarse": 1, "middle": 1, "fine": 3, "color": 4}
LOOKUP_BYTES = 8 * 32 * 4  # one trilinear lookup: 8 corner rows of 32 f32 channels


def algorithmic_per_point(stage, mode, fix_fine=False):
    """SURVEY.md §8(d)'s fixed convention, per sample point, per kernel: FLOP and HBM bytes.

    FLOP: forward = 2 MAC + trilinear (8 corners x 32 ch x 2 per lookup); dX = 2 MAC of the
    dX chains (the fine decoder's fc_c input gradient only for its own 32 grid channels:
    the middle features enter under no_grad, decoder.py:196-202) + trilinear backward (2x
    the forward trilinear per gradient lookup); dW = 2 MAC (BA mode).
    Bytes: forward = L_fwd lookups x 1,024 B; backward = per gradient lookup (each decoder
    samples its own grid with grad) the coordinate-gradient re-gather (1,024 B) plus, in BA
    mode, the grid-gradient scatter as a read-modify-write of the 8 corner rows (2 x 1,024 B);
    dW has no §8(d) bytes (its operands are the core's own intermediates).  At stage color,
    S = 48: 196,608 B/ray forward, 638,976 B/ray in BA mode -- SURVEY.md:461-462."""
    decs = STAGE_DECODERS[stage]
    ba = mode == "ba"
    lk_fwd, lk_grad = LOOKUPS_FWD[stage], len(decs)
    flop = {"k_mlp_fwd": 2 * sum(MAC[d] for d in decs) + TRI_FLOP * lk_fwd,
            "k_mlp_dx": 2 * sum(MAC_DX[d] for d in decs) + 2 * TRI_FLOP * lk_grad,
            "k_mlp_dw": 2 * sum(MAC[d] for d in decs if not fix_fine or d == "color") if ba else 0,
            "k_grid_gather": TRI_FLOP * LOOKUPS_UNIQUE[stage]}
    byt = {"k_mlp_fwd": LOOKUP_BYTES * lk_fwd,
           "k_mlp_dx": LOOKUP_BYTES * lk_grad * (3 if ba else 1),
           "k_mlp_dw": 0,
           "k_grid_gather": LOOKUP_BYTES * LOOKUPS_UNIQUE[stage]}
    return flop, byt


def step_roofline_rays_s(stage, S, mode, fix_fine=False):
    """§8(d) roofline rays/s of one GPU for the whole step (SURVEY.md:461-463): FLOP per ray =
    forward (2 MAC + trilinear) + dX (2 MAC) [+ dW (2 MAC), BA] + trilinear backward (2x the
    forward's); bytes per ray = the forward's and backward's lookups above; rays/s =
    min(f32 peak / FLOP, HBM peak / bytes).  Stage color, S = 48, BA: 15.17 MFLOP and
    638,976 B per ray -> 10.37 M rays/s."""
    decs = STAGE_DECODERS[stage]
    ba = mode == "ba"
    mac = sum(MAC[d] for d in decs)
    mac_dw = sum(MAC[d] for d in decs if not fix_fine or d == "color") if ba else 0
    tri = TRI_FLOP * LOOKUPS_FWD[stage]
    f_ray = S * (2 * mac + tri + 2 * mac + 2 * mac_dw + 2 * tri)
    _, byt = algorithmic_per_point(stage, mode, fix_fine)
    b_ray = S * (byt["k_mlp_fwd"] + byt["k_mlp_dx"])
    return min(FP32_MFMA_PEAK_TFLOPS * 1e12 / f_ray, HBM_PEAK_GBS * 1e9 / b_ray), f_ray, b_ray


# point-record geometry of the core (csrc/nc_mlp.hip Rec<KIND>): floats per point
REC_STRIDE = {"coarse": 368, "middle": 368, "fine": 400, "color": 368}
REC_LEN = {"coarse": 204, "middle": 204, "fine": 236, "color": 204}
FEAT = {"coarse": 32, "middle": 32, "fine": 64, "color": 32}
NOUT = {"coarse": 1, "middle": 1, "fine": 1, "color": 3}


def intermediate_bytes_per_point(stage, mode, jac=False, fix_fine=False):
    """Bytes per point each kernel moves through the core's OWN intermediates (activation
    records, point I/O, masks) -- not §8(d) algorithmic traffic, reported beside it
    (roofline.intermediate_bytes_per_launch).  k_mlp_fwd writes the forward record, k_mlp_dx
    reads masks / d out / coordinates and writes the backward record, k_mlp_dw streams both."""
    decs = STAGE_DECODERS[stage]
    ba = mode == "ba"
    wdw = [d for d in decs if not fix_fine or d == "color"] if ba else []  # decoders with dW
    fwd = sum(4 * FEAT[d] + 16 + 4 * (REC_LEN[d] - FEAT[d]) + 4 * NOUT[d] for d in decs)
    dx = sum(32 + 4 * NOUT[d] + 16 + 16 + 24 - (1024 - 384 if jac else 0) +
             (4 * (REC_STRIDE[d] - REC_LEN[d]) if d in wdw else 0) for d in decs)
    dw = sum(4 * REC_STRIDE[d] for d in wdw)  # (fourier_B's dW comes from k_mlp_dx: no dx in the record)
    gather = 128 * LOOKUPS_FWD[stage] + (384 * len(decs) if jac else 0)
    return {"k_mlp_fwd": fwd, "k_mlp_dx": dx, "k_mlp_dw": dw, "k_grid_gather": gather}


def samples_per_ray(args):
    """32 stratified + 16 surface samples with a gt depth; the coarse mapper (Mapper.py:600)
    and --render-depth none render without one: 32."""
    return 32 if (args.stage == "coarse" or args.render_depth == "none") else 48


def cpu_baseline(args, seconds):
    """The CPU oracle (torch-CPU restatement of the reference path) on a bounded sample."""
    from oracle import nice_oracle as O
    from nicecore import decoder as D
    from nicecore import scene as S
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or os.cpu_count()
    torch.set_num_threads(threads)
    sc = S.make_scene(args.scene)
    grids = S.init_grids(sc.shapes, generator=torch.Generator().manual_seed(0))
    m = D.build_default_nice(seed=0)
    prm = {k: v.detach().clone().requires_grad_(args.mode == "ba") for k, v in m.named_parameters()}
    g = {k: v.requires_grad_(args.mode == "ba") for k, v in grids.items()}
    dec_b = S.decoder_bounds(sc.bound)
    ro, rd, dep, col = S.synth_rays(sc, args.rays, seed=1000)
    kw = LOSS_KW[args.mode](args.stage)

    def it():
        for t in list(prm.values()) + list(g.values()):
            t.grad = None
        ro_ = ro.clone().requires_grad_(True)
        rd_ = rd.clone().requires_grad_(True)
        d, u, c = O.render_batch_ray(g, prm, dec_b, sc.bound, rd_, ro_, args.stage,
                                     dep if args.render_depth == "target" else None)
        if kw["loss"] == "mapper":
            loss = O.mapper_loss(d, c, dep, col, kw["w_color_loss"], kw["color_term"])
        else:
            loss = O.tracker_loss(d, u, c, dep, col, kw["w_color_loss"], True, True)
        loss.backward()

    it()  # warm-up
    n, t0 = 0, time.perf_counter()
    while True:
        it()
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds or n >= 50:
            break
    return {"value": args.rays * n / el, "unit": "rays/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model(),
            "sample": f"{n} iterations x {args.rays} rays x {samples_per_ray(args)} samples, stage {args.stage}, "
                      f"{args.mode} grads, torch CPU fp32/fp64 oracle, {threads} threads"}


def cpu_model() -> str:
    """The host CPU's model name (report the core count and CPU model)."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or platform.machine()


def read_traffic(args):
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3 --pmc
    summary (profiles/*traffic*.json) measured on this same workload, if present."""
    import glob
    want = traffic_config(args)
    # newest round first (profiles/r03/... sorts after profiles/r02/...)
    for fn in sorted(glob.glob(os.path.join(REPO, "profiles", "**", "*traffic*.json"), recursive=True), reverse=True):
        try:
            with open(fn) as f:
                d = json.load(f)
        except Exception:
            continue
        if d.get("config") == want:
            d["source"] = os.path.relpath(fn, REPO)
            return d
    return None


def traffic_config(args):
    """The workload key a PMC traffic summary is valid for (tools/pmc_traffic.py --config)."""
    return {"scene": args.scene, "rays": args.rays, "stage": args.stage, "mode": args.mode,
            "layout": args.layout, "fix_fine": bool(args.fix_fine), "render_depth": args.render_depth}


class _NullTimer:
    result = {}

    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def time_mapper_iteration(w, args):
    """render + loss + backward + Adam step (Mapper.py:590-625) as ONE graph replay:
    nicecore.optim.Adam(capturable=True) over the grids and decoder parameters."""
    from nicecore.graph import GraphedStep
    from nicecore.optim import Adam
    leaves = [g for g in w["grids"].values() if g.requires_grad] + \
        [p for p in w["model"].parameters() if p.requires_grad]
    opt = Adam(leaves, lr=1e-4, capturable=True)
    body = w["body"]

    def it():
        loss = body()
        opt.step()
        return loss
    g = GraphedStep(it)
    for _ in range(args.warmup):
        g()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        g()
    torch.cuda.synchronize()
    return round(1e3 * (time.perf_counter() - t0) / args.steps, 4)


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        launch_ranks(args)  # rank 0 prints the JSON line
        return
    world, rank, local = setup_dist(args)
    device = torch.device("cuda", torch.cuda.current_device())
    from nicecore import _lib as L
    L.load()
    w = build_workload(args, rank, device, world)
    eager, graphed = make_step(w, args, world, device)
    w["body"] = getattr(make_step, "last_body", None)
    for _ in range(args.warmup):
        eager()
    torch.cuda.synchronize()

    # per-kernel breakdown (separate eager pass, every library kernel event-timed on
    # its launch stream) -> dominant kernel and its average launch duration
    with L.KernelTimer() as kt_all:
        for _ in range(max(5, min(args.steps, 20))):
            eager()
    torch.cuda.synchronize()
    breakdown = {k: ms / n for k, (ms, n) in kt_all.result.items()}
    dominant = max(breakdown, key=breakdown.get)

    # eager step time (reported beside the graph-replay value)
    t0 = time.perf_counter()
    for _ in range(max(5, min(args.steps, 20))):
        eager()
    torch.cuda.synchronize()
    eager_ms = 1e3 * (time.perf_counter() - t0) / max(5, min(args.steps, 20))
    # the same eager step with the other parameter-gradient mode (reported beside it)
    other = "direct" if args.param_grads == "autograd" else "autograd"
    w["renderer"].param_grads = other
    for _ in range(3):
        eager()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(max(5, min(args.steps, 20))):
        eager()
    torch.cuda.synchronize()
    eager_other_ms = 1e3 * (time.perf_counter() - t0) / max(5, min(args.steps, 20))
    w["renderer"].param_grads = args.param_grads

    step = graphed if graphed is not None else eager
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    import torch.distributed as dist
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    timer = L.KernelTimer([dominant]) if graphed is None else _NullTimer()
    with timer as kt:  # eager: 2 event records per step around the kernel, on its launch stream
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    dt = torch.tensor([t1 - t0], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    dt = float(dt.item())
    if graphed is None:
        ms_dom, n_dom = kt.result.get(dominant, (0.0, 0))
        timing_src = f"HIP events on the launch stream, {n_dom} launches in the timed region"
    else:  # events inside a replayed graph keep only the last replay: use the eager pass
        ms_dom, n_dom = kt_all.result.get(dominant, (0.0, 0))
        timing_src = (f"HIP events on the launch stream, {n_dom} launches of the same step run "
                      f"eagerly just before the graph-replay timed region")
    avg_ms = ms_dom / max(n_dom, 1)

    S = samples_per_ray(args)
    from nicecore import render_fn as RF
    flop_pt, byte_pt = algorithmic_per_point(args.stage, args.mode, args.fix_fine)
    inter_pt = intermediate_bytes_per_point(args.stage, args.mode, jac=RF._SAVE_JAC, fix_fine=args.fix_fine)
    points = args.rays * S  # units one launch processes
    roof = None
    if dominant in flop_pt and avg_ms > 0:
        fl = flop_pt[dominant] * points
        by = byte_pt[dominant] * points
        t = avg_ms * 1e-3
        tflops = fl / t / 1e12
        gbs = by / t / 1e9
        mpeak = MFMA_PEAK.get(dominant, FP32_MFMA_PEAK_TFLOPS)
        ridge = mpeak * 1e12 / (HBM_PEAK_GBS * 1e9)  # FLOP per byte
        tr = read_traffic(args)
        kt_pmc = (tr or {}).get("kernels", {}).get(dominant) or {}
        traffic = kt_pmc.get("hbm_bytes")
        atomic = kt_pmc.get("atomic_bytes")  # PMC TCC_EA0_ATOMIC x 64 B, same workload
        # the limiter = the highest of the fractions: HBM (SURVEY §8(d) bytes), MFMA (algorithmic
        # FLOP) and, where the PMC summary has it, the memory-side float-atomic path
        fracs = {"hbm": gbs / HBM_PEAK_GBS, "mfma": tflops / mpeak}
        if atomic:
            fracs["atomic"] = atomic / t / 1e9 / ATOMIC_PEAK_GBS
        bound = max(fracs, key=fracs.get)
        ach = {"hbm": gbs, "mfma": tflops, "atomic": (atomic or 0) / t / 1e9}[bound]
        roof = {"bound": bound, "kernel": dominant,
                "achieved": round(ach, 3),
                "peak": {"hbm": HBM_PEAK_GBS, "mfma": mpeak, "atomic": ATOMIC_PEAK_GBS}[bound],
                "unit": "TFLOP/s" if bound == "mfma" else "GB/s",
                "frac": round(fracs[bound], 4),
                "traffic": traffic,
                "traffic_source": (tr or {}).get("source"),
                "traffic_frac": round(traffic / t / 1e9 / HBM_PEAK_GBS, 4) if traffic else None,
                "avg_launch_ms": round(avg_ms, 4),
                "points_per_launch": points,
                "bytes_per_point": byte_pt[dominant], "flop_per_point": flop_pt[dominant],
                "bytes_per_launch": by, "flop_per_launch": fl,
                "bytes_convention": "SURVEY.md §8(d): 1,024 B per trilinear lookup read; grid-gradient "
                                    "scatter = read-modify-write of the 8 corner rows (2 x 1,024 B)",
                "intermediate_bytes_per_launch": inter_pt.get(dominant, 0) * points,
                "intensity_flop_per_byte": round(fl / by, 2) if by else None,
                "ridge_flop_per_byte": round(ridge, 2),
                "mfma_tflops": round(tflops, 3), "mfma_peak_tflops": round(mpeak, 1),
                "mfma_frac": round(tflops / mpeak, 4),
                "hbm_gbs": round(gbs, 1), "hbm_frac": round(gbs / HBM_PEAK_GBS, 4),
                "atomic_bytes": atomic, "atomic_gbs": round(atomic / t / 1e9, 1) if atomic else None,
                "atomic_peak_gbs": ATOMIC_PEAK_GBS,
                "atomic_frac": round(fracs["atomic"], 4) if atomic else None,
                "timing": timing_src}
    peak_rays, f_ray, b_ray = step_roofline_rays_s(args.stage, S, args.mode, args.fix_fine)

    total_rays = args.global_rays or world * args.rays  # rays all ranks render per step
    value = total_rays * args.steps / dt
    out = {
        "metric": METRIC, "value": round(value, 1), "unit": "rays/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * dt / args.steps, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "gemm": "decoder GEMMs of k_mlp_fwd as split-f16 MFMA (3 x f16, f32 accumulate, error at or "
                "below the f32 MFMA's: tools/split16_bench.hip); k_mlp_dx/k_mlp_dw exact f32 MFMA; "
                "sampling/compositing f64",
        "data": "synthetic",
        "config": {"workload": f"{args.scene} {args.rays} rays x {S} samples per GPU, stage {args.stage}, "
                               f"{'mapper/BA grads (rays+grids+decoders)' if args.mode == 'ba' else 'tracker grads (rays)'}"
                               f"{', fix_fine: color-decoder dW only' if args.fix_fine else ''}",
                   "rays_per_gpu": args.rays, "samples_per_ray": S, "stage": args.stage,
                   "mode": args.mode, "grid_layout": args.layout, "parallelism": f"dp{world}",
                   "grid_grads": "sparse rows" if w["sparse"] is not None else "dense",
                   "grid_exchange": (None if world == 1 else "sparse row union" if w["sparse"] is not None else
                                     "dense" if w["frustum"] is None else
                                     "frustum rows (Mapper frustum_feature_selection): %d of %d voxels" % (
                                         sum(int(v.numel()) for v in w["frustum"].values()),
                                         sum(int(w["grids"][k][0, 0].numel()) for k in w["frustum"]))),
                   "overlap": "grid all-reduce beside k_mlp_dw" if (w["ba"] and w["sparse"] is None and (
                       args.overlap == "on" or (args.overlap == "auto" and world > 1))) else "none"},
        "roofline": roof,
        "step_roofline": {"rays_s_per_gpu_peak": round(peak_rays), "flop_per_ray": f_ray, "bytes_per_ray": b_ray,
                          "frac": round(value / world / peak_rays, 4),
                          "note": "SURVEY.md §8(d): min(157.3 TF / FLOP per ray, 8 TB/s / bytes per ray)"},
        "launch": "hipGraph replay" if graphed is not None else "eager",
        "eager_ms_per_step": round(eager_ms, 4),
        "param_grads": args.param_grads,
        f"eager_{other}_ms_per_step": round(eager_other_ms, 4),
        "kernels_ms": {k: round(v, 4) for k, v in sorted(breakdown.items(), key=lambda kv: -kv[1])},
    }
    if args.dump_grads:
        eager()  # one more step: render + loss + backward + the gradient exchange
        torch.cuda.synchronize()
        if rank == 0:
            dump = {"world": world, "rays_per_rank": args.rays, "total_rays": total_rays,
                    "params": {n: p.grad.detach().cpu() for n, p in w["model"].named_parameters()
                               if p.grad is not None}, "grids": {}}
            for k, g in w["grids"].items():
                if g.grad is None:
                    continue
                flat = g.grad.detach()[0].reshape(g.shape[1], -1)  # [C, D*H*W]
                rows = (w["frustum"] or {}).get(k)
                dump["grids"][k] = (flat[:, rows] if rows is not None else flat).cpu()
            if w["frustum"] is not None:
                dump["frustum_rows"] = {k: v.cpu() for k, v in w["frustum"].items()}
            torch.save(dump, args.dump_grads)
    if args.iteration and world == 1 and w["ba"] and w["sparse"] is None:
        out["mapper_iteration_ms"] = time_mapper_iteration(w, args)
    if world == 1 and rank == 0 and args.cpu_seconds > 0:
        from nicecore import scene as S_
        if S_.grids_bytes(S_.make_scene(args.scene).shapes) > (8 << 30):
            out["cpu_baseline"] = {"value": None, "unit": "rays/s", "cores": None, "kind": "port",
                                   "sample": "not run: the scene's grids do not fit a bounded CPU sample"}
        else:
            out["cpu_baseline"] = cpu_baseline(args, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
