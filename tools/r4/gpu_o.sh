#!/bin/bash
# round 4 session o: scatter staging without spill reloads (lane ids recomputed, scalar slice base): parity suites + bench
# the NICE_CORE_PROFILE test: the scatter / parity / sparse / configs suites
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4o
mkdir -p $O
step() { # name seconds cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "[$n] rc=$rc"; tail -4 $O/$n.log | cut -c1-400
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sparse.py tests/test_gpu_configs.py tests/test_gpu_loss.py tests/test_initstd.py tests/test_gpu_dense_accumulate.py tests/test_gpu_jacobian.py tests/test_gpu_ray_mask.py tests/test_gpu_defer.py -m gpu -x -q --timeout 300 --timeout-method thread
step bench 300 python3 -u bench.py
