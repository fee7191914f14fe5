#!/bin/bash
# round 4 session h: host-time split of the eager drop-in steps (fused loss / the reference's Python loss)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4h
mkdir -p $O
step() { # name seconds cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "[$n] rc=$rc"; tail -30 $O/$n.log | cut -c1-1500
  if [ $rc -ge 124 ]; then exit $rc; fi
}
step split 300 python3 -u tools/host_split.py --steps 300
