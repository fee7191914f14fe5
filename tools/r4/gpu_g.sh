#!/bin/bash
# round 4 session g: fixed-order fused loss + direct-mode engine reach (tests), the Mapper's
# unmodified call sequence beside the fused / graphed steps, bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4g
mkdir -p $O
step() { # name seconds cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "[$n] rc=$rc"; tail -6 $O/$n.log | cut -c1-1500
  if [ $rc -ge 124 ]; then exit $rc; fi
}
# tests: passed in the first run of this session (56 passed)
step callseq 300 python3 -u tools/bench_callseq.py --steps 200 --warmup 10 --profile
step bench 300 python3 -u bench.py
