#!/bin/bash
# round 3 session c: counter list, rocprofv3 stats + HBM traffic + SQ passes of the C2 bench
cd "$(dirname "$0")/.."
ROOT=$(pwd)
export TMPDIR=/tmp
O=$ROOT/gpurun_out/r3c
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_determinism.py tests/test_gpu_sparse.py > $O/tests_det.log 2>&1
rc=$?; echo "det tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
NC_DETERMINISTIC=1 timeout -k 10 300 python -u bench.py --cpu-seconds 0 > $O/bench_c2_det.log 2>&1
rc=$?; echo "det bench rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
(cd /tmp && timeout -s KILL 120 rocprofv3 -L > $O/counters.txt 2>&1); echo "list rc=$?"
for c in SQ_INSTS_VALU_MFMA_F16 SQ_INSTS_VALU_MFMA_F32 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES; do
  if grep -q "$c" $O/counters.txt; then echo "have $c"; else echo "MISSING $c"; fi
done
./tools/prof_session.sh r3c --steps 20 > $O/prof.log 2>&1
rc=$?; echo "prof rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
./tools/pmc_session.sh r3c --steps 10 > $O/pmc.log 2>&1
rc=$?; echo "pmc rc=$rc"
python3 tools/pmc_report.py gpurun_out/pmc_r3c > $O/pmc_sq.txt 2>&1
echo "report rc=$?"
