#!/bin/bash
# round 4 session q: the gradient zero fill on a forked stream beside the forward (NICECORE_FILL_FORK A/B), tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4q
mkdir -p $O
step() { # name seconds cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "[$n] rc=$rc"; tail -2 $O/$n.log | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_loss.py tests/test_gpu_grad_pool.py tests/test_gpu_defer.py tests/test_gpu_ray_mask.py tests/test_initstd.py tests/test_gpu_sparse.py tests/test_gpu_determinism.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread
for i in 1 2 3; do
  NICECORE_FILL_FORK=0 step base$i 200 python3 -u bench.py --steps 200 --warmup 20 --cpu-seconds 0
  NICECORE_FILL_FORK=1 step fork$i 200 python3 -u bench.py --steps 200 --warmup 20 --cpu-seconds 0
done
for f in $O/base*.log $O/fork*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f) $(grep -o '"kernels_ms": {[^}]*}' $f)"; done
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 50 --warmup 5 --cpu-seconds 0
