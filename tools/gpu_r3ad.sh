#!/bin/bash
# round 3 session ad: trilinear backward split out of k_mlp_dx into k_grid_bwd
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r3ad
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/tests_all.log 2>&1
rc=$?; echo "all tests rc=$rc"; tail -2 $O/tests_all.log; grep FAILED $O/tests_all.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for v in 0 1 0 1; do
  NICECORE_SPLIT_TRI=$v timeout -k 10 120 python -u bench.py --cpu-seconds 0 > $O/bench_split$v.log 2>&1
  rc=$?; echo "bench split=$v rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
  grep -o '"ms_per_step": [0-9.]*\|"kernels_ms": {[^}]*}' $O/bench_split$v.log
done
