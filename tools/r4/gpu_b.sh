#!/bin/bash
# round 4 session b: init-std parity + ray mask tests, whole GPU suite, bench line, tracker iteration
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4b
mkdir -p $O
step() { # name seconds cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "[$n] rc=$rc"; tail -4 $O/$n.log
  if [ $rc -ge 124 ]; then exit $rc; fi
}
step tests_new 500 python3 -u -m pytest tests/test_initstd.py tests/test_gpu_ray_mask.py tests/test_gpu_loss.py tests/test_gpu_bench_ranks.py -m gpu -v --timeout 300 --timeout-method thread
step bench_c2 300 python3 -u bench.py --steps 20 --warmup 5
step tracker_iter 300 python3 -u tools/bench_tracker_iteration.py --graph
step tests_all 900 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread
step prof 900 tools/prof_session.sh r4b --steps 20 --warmup 5
