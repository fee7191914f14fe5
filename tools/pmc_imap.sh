#!/bin/bash
# SQ counter passes (<= 8 SQ counters each) over tools/bench_imap.py (iMAP* Mapper iteration).
#   tools/pmc_session.sh <tag> [bench args...]
tag="$1"; shift
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
out="$ROOT/gpurun_out/pmc_imap_$tag"
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
export HSA_ENABLE_IPC_MODE_LEGACY=0
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VALU_MFMA_F32"
B="SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM SQ_WAVES GRBM_GUI_ACTIVE"
# f16 MFMA instructions (k_mlp_fwd's split-f16 GEMMs) and the MFMA busy cycles again with the
# kernel's clock count in the same pass (GRBM_GUI_ACTIVE: summed over the 8 XCDs)
C="SQ_INSTS_VALU_MFMA_F16 SQ_INSTS_VALU_MFMA_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
n=0
for set in "$A" "$B" "$C"; do
  n=$((n+1))
  echo "=== pass $n: $set"
  timeout -s KILL 300 rocprofv3 --pmc $set --kernel-include-regex "nc::" --output-format csv -d "$out/p$n" -o run -- \
      python3 "$ROOT/tools/bench_imap.py" --steps 2 --warmup 1 "$@" > "$out/p$n.log" 2>&1
  rc=$?; echo "=== pass $n rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
