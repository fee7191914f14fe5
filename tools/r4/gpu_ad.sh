#!/bin/bash
# round 4 session ad: k_param_ray_reduce with 4 / 8 / 12 slab rows in flight per thread
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4ad
mkdir -p $O
step() { # name seconds cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "[$n] rc=$rc"; tail -8 $O/$n.log | cut -c1-200
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_determinism.py tests/test_gpu_grad_pool.py -m gpu -x -q --timeout 300 --timeout-method thread
step ab 500 python3 -u tools/ablate.py run cur pr4 pr12 cur pr4 pr12 cur pr4
