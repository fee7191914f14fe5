#!/bin/bash
# round 4 session j: k_mlp_dw ablations on the current tree; the caller-only share of the
# Mapper's unmodified call sequence
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4j
mkdir -p $O
step() { # name seconds cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "[$n] rc=$rc"; tail -12 $O/$n.log | cut -c1-600
  if [ $rc -ge 124 ]; then exit $rc; fi
}
step ab 600 python3 -u tools/ablate.py run cur dw_no_mfma dw_no_stage dw_no_emb dw_no_maskpass dw_no_load dw_none cur
step callseq 300 python3 -u tools/bench_callseq.py --steps 200 --warmup 10
