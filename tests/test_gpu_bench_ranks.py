"""bench.py's N > 1 path, run as the driver runs it (a fresh process per call), on one GPU:
two or three ranks over gloo (bench.launch_ranks spawns them; RCCL needs one GPU per rank)
against one rank, on the SAME global batch (--global-rays: rank r renders its contiguous
shard of the rays the single rank renders, distributed.shard_bounds -- with 3 ranks the
shards are uneven, 334 / 333 / 333), on Replica room0 and on Apartment (C4).

One step after the timed ones (--dump-grads) is compared: the exchanged gradients of the
two ranks -- the frustum rows of the three grids (the Mapper's frustum_feature_selection,
Mapper.py:371-414, exchanged by distributed.allreduce_rows_async) and every decoder
parameter -- must equal the single rank's to 1e-5 of each tensor's max-abs (the sums differ
only in their float association), with and without the DeferParamGrads overlap (the grid
all-reduce beside k_mlp_dw).  The batch-global max(gt_depth) is all-reduced before the
render (Renderer.py:157, :194), so the shards sample exactly as the whole batch does."""
import json
import os
import subprocess
import sys

import pytest
import torch

from conftest import REPO
from parity_common import rel_err


def _bench(tmp_path, name, *args):
    out = tmp_path / f"{name}.pt"
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, "-u", os.path.join(REPO, "bench.py"), "--steps", "3", "--warmup", "2",
                        "--cpu-seconds", "0", "--frustum", "on", "--dump-grads", str(out), *args],
                       capture_output=True, text=True, timeout=400, env=env, cwd=REPO)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    return line, torch.load(out, weights_only=True)


_ONE = {}


def _one_rank(tmp_path, scene, total):
    """The single-rank reference of a (scene, total rays) batch, run once per module."""
    key = (scene, total)
    if key not in _ONE:
        _ONE[key] = _bench(tmp_path, f"one_{scene}_{total}", "--gpus", "1", "--scene", scene,
                           "--global-rays", str(total), "--overlap", "off")
    return _ONE[key]


def _check_equal(one, two, world, total):
    from nicecore.distributed import shard_bounds
    assert two["world"] == world and one["world"] == 1
    assert two["total_rays"] == one["total_rays"] == total
    a, b = shard_bounds(total, 0, world)
    assert two["rays_per_rank"] == b - a  # rank 0's shard (the larger one when uneven)
    for k in one["frustum_rows"]:
        assert torch.equal(one["frustum_rows"][k], two["frustum_rows"][k]), k
    assert set(one["grids"]) == set(two["grids"]) and len(one["grids"]) == 3
    assert set(one["params"]) == set(two["params"]) and len(one["params"]) > 0
    bad = {}
    for group in ("grids", "params"):
        for k, ref in one[group].items():
            e = rel_err(two[group][k], ref)
            if not e <= 1e-5:
                bad[f"{group}/{k}"] = e
    assert not bad, bad


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("overlap", ["on", "off"])
def test_gloo_ranks_equal_one_rank(tmp_path, world, overlap):
    """world 2 (500 + 500 rays) and world 3 (334 + 333 + 333: distributed.shard_bounds'
    remainder) on one 1,000-ray Replica room0 batch."""
    one_line, one = _one_rank(tmp_path, "replica_room0", 1000)
    line, many = _bench(tmp_path, f"w{world}_{overlap}", "--gpus", str(world), "--backend", "gloo",
                        "--global-rays", "1000", "--overlap", overlap)
    assert one_line["n_gpus"] == 1 and line["n_gpus"] == world
    assert line["config"]["parallelism"] == f"dp{world}"
    assert line["config"]["grid_exchange"].startswith("frustum rows")
    assert line["config"]["overlap"] == ("grid all-reduce beside k_mlp_dw" if overlap == "on" else "none")
    _check_equal(one, many, world, 1000)


@pytest.mark.gpu
def test_gloo_ranks_apartment_frustum_rows(tmp_path):
    """Apartment (BASELINE C4 geometry: 625 rays per GPU of a 5,000-ray window): two ranks of
    625 rays with the frustum-row exchange against one rank of the 1,250-ray batch."""
    one_line, one = _one_rank(tmp_path, "apartment", 1250)
    line, two = _bench(tmp_path, "apartment_w2", "--gpus", "2", "--backend", "gloo", "--scene", "apartment",
                       "--global-rays", "1250", "--overlap", "auto")
    assert line["n_gpus"] == 2 and line["config"]["rays_per_gpu"] == 625
    assert line["config"]["grid_exchange"].startswith("frustum rows")
    _check_equal(one, two, 2, 1250)


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_gloo_ranks_c4_apartment_world8(tmp_path):
    """BASELINE C4 as stated: Apartment, one 5,000-ray window (40 keyframes x 125 rays,
    synth_rays' 40 poses), 8 ranks of 625 rays (gloo, on this one GPU), the frustum-row
    exchange with the grid all-reduce beside k_mlp_dw (overlap on): the rank-summed
    frustum-row and decoder gradients equal one rank's 5,000-ray step to 1e-5 of max-abs."""
    one_line, one = _one_rank(tmp_path, "apartment", 5000)
    line, eight = _bench(tmp_path, "apartment_w8", "--gpus", "8", "--backend", "gloo", "--scene", "apartment",
                         "--global-rays", "5000", "--overlap", "on")
    assert line["n_gpus"] == 8 and line["config"]["rays_per_gpu"] == 625
    assert line["config"]["parallelism"] == "dp8"
    assert line["config"]["grid_exchange"].startswith("frustum rows")
    assert line["config"]["overlap"] == "grid all-reduce beside k_mlp_dw"
    _check_equal(one, eight, 8, 5000)
