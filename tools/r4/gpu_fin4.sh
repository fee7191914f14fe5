#!/bin/bash
# round 4 closing session 4 (after the scatter preload and register scan): full GPU suite, smoke, the
# default and NC_DETERMINISTIC bench lines, rocprofv3 stats + HBM / atomic counters of C2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4fin4
mkdir -p $O
step() { # name seconds cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "[$n] rc=$rc"; tail -3 $O/$n.log | cut -c1-400
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smoke 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench 300 python3 -u bench.py
NC_DETERMINISTIC=1 step bench_det 300 python3 -u bench.py

