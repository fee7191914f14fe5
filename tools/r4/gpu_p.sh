#!/bin/bash
# round 4 evidence session p (after the spill-free scatter staging): full GPU suite, smoke, the default bench line, rocprofv3
# stats + HBM / atomic counters of the C2 bench, the other configs, the masked tracker
# iteration, the Mapper call-sequence comparison
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4p
mkdir -p $O
step() { # name seconds cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "[$n] rc=$rc"; tail -4 $O/$n.log | cut -c1-600
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smoke 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench 300 python3 -u bench.py
step prof 900 bash tools/prof_session.sh r4p --steps 20 --warmup 5
step configs 900 bash tools/configs_session.sh r4p
step tracker_it 300 python3 -u tools/bench_tracker_iteration.py --graph
step callseq 300 python3 -u tools/bench_callseq.py --steps 200 --warmup 10
