"""bench.py's N > 1 path, run as the driver runs it (a fresh process per call), on one GPU:
two ranks over gloo (bench.launch_ranks spawns them; RCCL needs one GPU per rank) against
one rank, on the SAME global batch (--global-batch: rank r renders its contiguous shard of
the 1,000 rays the single rank renders, distributed.shard).

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
                        "--cpu-seconds", "0", "--global-batch", "--frustum", "on", "--dump-grads", str(out), *args],
                       capture_output=True, text=True, timeout=400, env=env, cwd=REPO)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    return line, torch.load(out, weights_only=True)


@pytest.mark.gpu
@pytest.mark.parametrize("overlap", ["on", "off"])
def test_two_gloo_ranks_equal_one_rank(tmp_path, overlap):
    one_line, one = _bench(tmp_path, "one", "--gpus", "1", "--rays", "1000", "--overlap", overlap)
    two_line, two = _bench(tmp_path, "two", "--gpus", "2", "--backend", "gloo", "--rays", "500", "--overlap", overlap)
    assert one_line["n_gpus"] == 1 and two_line["n_gpus"] == 2
    assert two_line["config"]["parallelism"] == "dp2" and two_line["config"]["rays_per_gpu"] == 500
    assert two_line["config"]["grid_exchange"].startswith("frustum rows")
    assert two_line["config"]["overlap"] == ("grid all-reduce beside k_mlp_dw" if overlap == "on" else "none")
    assert two["world"] == 2 and one["world"] == 1
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
