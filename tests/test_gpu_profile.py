"""NICE_CORE_PROFILE=1 (SURVEY.md §5 "tracing"): every kernel launch of the core is timed
with HIP events on its launch stream and a per-kernel table is printed to stderr at exit
(nc_profile_report, registered by nicecore._lib.load); launches enqueued while a stream is
being captured into a graph are counted apart, not timed.  Run as the bench runs, in a
fresh process."""
import json
import os
import re
import subprocess
import sys

import pytest

from conftest import REPO


@pytest.mark.gpu
def test_profile_report_at_exit():
    env = dict(os.environ, NICE_CORE_PROFILE="1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, "-u", os.path.join(REPO, "bench.py"), "--steps", "3", "--warmup", "2",
                        "--rays", "200", "--cpu-seconds", "0"], capture_output=True, text=True, timeout=300,
                       env=env, cwd=REPO)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["ms_per_step"] > 0
    err = r.stderr
    assert "[NICE_CORE_PROFILE] per-kernel HIP-event times" in err, err[-3000:]
    rows = {m.group(1): (int(m.group(2)), float(m.group(3)))
            for m in re.finditer(r"^\s+(k_\w+)\s+(\d+)\s+([\d.]+)\s+[\d.]+\s+[\d.]+%$", err, re.M)}
    for k in ("k_ray_setup", "k_mlp_fwd", "k_mlp_dx", "k_mlp_dw"):
        assert k in rows and rows[k][0] > 0 and rows[k][1] > 0.0, (k, rows)
    # the timed region replays a captured graph: its launches are reported apart
    assert "launches enqueued during graph capture" in err
