#!/bin/bash
# k_param_ray_reduce rows in flight (NC_PR_DEPTH) A/B + the parity / determinism tests that
# read the reduced parameter gradients
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/am
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_determinism.py tests/test_gpu_loss.py > $O/tests.log 2>&1 &&
timeout -k 10 400 python -u tools/ablate.py run cur pr4 pr8 pr16 cur pr4 pr8 pr16 > $O/ab_pr_depth.log 2>&1
