#!/bin/bash
# round 4 session l: split-f16 k_mlp_dw (parity tests, then A/B against the f32 dW build)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4l
mkdir -p $O
step() { # name seconds cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "[$n] rc=$rc"; tail -12 $O/$n.log | cut -c1-400
  if [ $rc -ge 124 ]; then exit $rc; fi
}
step tests 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_initstd.py tests/test_gpu_loss.py tests/test_gpu_grad_pool.py tests/test_gpu_defer.py tests/test_gpu_ray_mask.py -m gpu -x -q --timeout 300 --timeout-method thread
step ab 600 python3 -u tools/ablate.py run dwf32 cur dwf32 cur
