#!/bin/bash
# round 4 session e: A/B of the index-arithmetic changes (global zero row) against the round's base library
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4e
mkdir -p $O
step() { # name seconds cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "[$n] rc=$rc"; tail -6 $O/$n.log | cut -c1-1500
  if [ $rc -ge 124 ]; then exit $rc; fi
}
step ab 600 python3 -u tools/ablate.py run r4base r4cur r4base r4cur
step tests_core 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_initstd.py tests/test_gpu_ray_mask.py tests/test_gpu_configs.py tests/test_gpu_loss.py -m gpu -q --timeout 300 --timeout-method thread
