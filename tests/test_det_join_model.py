"""The ordered grid scatter's run summation as nc_det.hip implements it (k_det_runs'
16-entry sub-chunks, the in-chunk join of runs crossing sub-chunks, k_det_join across
chunks), modelled in Python (tools/det_join_sim.py) and checked against a segmented sum:
every voxel key written exactly once, with its sum, for random run-length patterns.
The GPU kernels themselves are checked bit-for-bit run to run and against the oracle in
tests/test_gpu_determinism.py."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import det_join_sim  # noqa: E402


def test_run_join_model_writes_every_voxel_once():
    det_join_sim.check(trials=120, seed=3)
