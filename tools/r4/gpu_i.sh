#!/bin/bash
# round 4 session i: gradient zero fill in k_composite_fwd_loss's spare workgroups (A/B by env), tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4i
mkdir -p $O
step() { # name seconds cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "[$n] rc=$rc"; tail -3 $O/$n.log | cut -c1-400
  if [ $rc -ge 124 ]; then exit $rc; fi
}
step tests 600 python3 -u -m pytest tests/test_gpu_loss.py tests/test_gpu_grad_pool.py tests/test_gpu_parity.py tests/test_initstd.py tests/test_gpu_range_guard.py -m gpu -q --timeout 300 --timeout-method thread
for i in 1 2 3; do
  NICECORE_FILL_IN_COMPOSITE=0 step base$i 200 python3 -u bench.py --steps 200 --warmup 20 --cpu-seconds 0
  NICECORE_FILL_IN_COMPOSITE=1 step new$i 200 python3 -u bench.py --steps 200 --warmup 20 --cpu-seconds 0
done
grep -ho '"ms_per_step": [0-9.]*' $O/base*.log $O/new*.log
step prof 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u bench.py --steps 50 --warmup 5 --cpu-seconds 0
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cut -d, -f1-4 {} | head -9
