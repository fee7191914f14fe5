#!/bin/bash
# round 4 session c: int32 corner indexing -- full GPU suite, bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4c
mkdir -p $O
step() { # name seconds cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "[$n] rc=$rc"; tail -4 $O/$n.log
  if [ $rc -ge 124 ]; then exit $rc; fi
}
step bench_c2 300 python3 -u bench.py --steps 20 --warmup 5 --cpu-seconds 0
step tests_all 1000 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
step bench_c2_2 300 python3 -u bench.py --steps 20 --warmup 5 --cpu-seconds 0
