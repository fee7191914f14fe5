#!/bin/bash
# round 4 session n: k_mlp_dx with the tile's p.float() and coordinates parked in LDS at the tile start (park) against the committed build (lane)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4n
mkdir -p $O
step() { # name seconds cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "[$n] rc=$rc"; tail -12 $O/$n.log | cut -c1-400
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step ab 600 python3 -u tools/ablate.py run lane park lane park lane park
