#!/bin/bash
# round 3 session v: grid scatter moved from k_mlp_dx into workgroups of the k_mlp_dw launch.
# Parity (whole GPU suite) first, then A/B of the step against the inline scatter.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r3v
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/tests_all.log 2>&1
rc=$?; echo "all tests rc=$rc"; tail -2 $O/tests_all.log
if [ $rc -ne 0 ]; then exit $rc; fi
for v in inline 32 16 24 48 64 inline 32; do
  if [ "$v" = inline ]; then e="NICECORE_SCATTER=inline"; else e="NICECORE_SCAT_WGS=$v"; fi
  env $e timeout -k 10 120 python -u bench.py --cpu-seconds 0 > $O/bench_$v.log 2>&1
  rc=$?; echo "bench $v rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
  grep -o '"ms_per_step": [0-9.]*\|"kernels_ms": {[^}]*}' $O/bench_$v.log
done
