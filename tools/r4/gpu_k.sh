#!/bin/bash
# round 4 session k: the gradient zero fill split between k_ray_setup's and
# k_composite_fwd_loss's extra workgroups (NICECORE_FILL_SETUP_PCT sweep), tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4k
mkdir -p $O
step() { # name seconds cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "[$n] rc=$rc"; tail -2 $O/$n.log | cut -c1-300
  if [ $rc -ge 124 ]; then exit $rc; fi
}
step tests 600 python3 -u -m pytest tests/test_gpu_loss.py tests/test_gpu_grad_pool.py tests/test_gpu_parity.py tests/test_initstd.py tests/test_gpu_ray_mask.py tests/test_gpu_defer.py -m gpu -q --timeout 300 --timeout-method thread
for i in 1 2; do
  for p in fwd 0 30 50 70 100; do
    NICECORE_FILL_SETUP_PCT=$p step b_${p}_$i 200 python3 -u bench.py --steps 200 --warmup 20 --cpu-seconds 0
  done
done
for f in $O/b_*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f) $(grep -o '"kernels_ms": {[^}]*}' $f)"; done
