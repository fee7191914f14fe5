#!/bin/bash
# round 4 session s: k_det_runs without scratch (runs written RG at a time) -- determinism
# tests, the NC_DETERMINISTIC bench line and its kernel stats
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4s
mkdir -p $O
step() { # name seconds cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "[$n] rc=$rc"; tail -2 $O/$n.log | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step det_tests 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_determinism.py
NC_DETERMINISTIC=1 step bench 300 python3 -u bench.py --steps 50 --warmup 5 --cpu-seconds 0
NC_DETERMINISTIC=1 step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 "$f" | head -20
