#!/bin/bash
# round 4 session ag: k_det_runs runs per write-back group 4 / 8 / 16
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4ag
mkdir -p $O
step() { # name seconds cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "[$n] rc=$rc"; tail -7 $O/$n.log | cut -c1-130
  if [ $rc -ne 0 ]; then exit $rc; fi
}
NC_DETERMINISTIC=1 step ab 400 python3 -u tools/ablate.py run cur det_rg4 det_rg16 cur det_rg4 det_rg16
