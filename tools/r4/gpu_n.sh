#!/bin/bash
# round 4 session n: zero-fill workgroups per CU in k_composite_fwd_loss (1, 2, 3)
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
step ab 600 python3 -u tools/ablate.py run cur fill2 fill3 cur fill2 fill3
