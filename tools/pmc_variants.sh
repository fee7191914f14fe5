#!/bin/bash
# One SQ counter pass per library variant (dbg/abl_<variant>.so, tools/ablate.py build) over the
# eager C2 bench step, restricted to one kernel: VALU / MFMA / LDS instruction counts per variant
# (the attribution table of an ablation study).  Run from the repo root on the GPU box.
#   tools/pmc_variants.sh <tag> <kernel-regex> <variant>... [-- bench args]
tag="$1"; krx="$2"; shift 2
vars=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do vars+=("$1"); shift; done
[ "$1" = "--" ] && shift
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
out="$ROOT/gpurun_out/$tag"
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
C1="SQ_INSTS_VALU SQ_INSTS_VALU_MFMA_F16 SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
C2="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_WAVES"
C3="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES"
for v in "${vars[@]}"; do
  lib="$ROOT/dbg/abl_$v.so"
  [ -f "$lib" ] || { echo "missing $lib"; exit 2; }
  n=0
  for C in "$C1" "$C2" "$C3"; do
    n=$((n+1))
    echo "=== $v pass $n"
    NICECORE_LIB="$lib" timeout -s KILL 240 rocprofv3 --pmc $C --kernel-include-regex "$krx" --output-format csv \
        -d "$out/$v/p$n" -o run -- python3 "$ROOT/bench.py" --eager --steps 5 --warmup 2 --cpu-seconds 0 "$@" \
        > "$out/$v.p$n.log" 2>&1
    rc=$?; echo "=== $v pass $n rc=$rc"
    [ $rc -ne 0 ] && { tail -5 "$out/$v.p$n.log"; exit $rc; }
  done
  python3 "$ROOT/tools/pmc_report.py" "$out/$v" | tee "$out/$v.txt"
done
exit 0
