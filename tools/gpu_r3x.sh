#!/bin/bash
# scatter-waves ablation: dW with 12 waves + idle scatter waves (2), staged without atomics (3), full (1)
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r3x
mkdir -p $O
for v in inline 2 3 1; do
  if [ "$v" = inline ]; then e="NICECORE_SCATTER=inline"; else e="NICECORE_SCAT_ABL=$v"; fi
  env $e timeout -k 10 120 python -u bench.py --cpu-seconds 0 > $O/bench_$v.log 2>&1
  rc=$?; echo "bench $v rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
  grep -o '"ms_per_step": [0-9.]*\|"kernels_ms": {[^}]*}' $O/bench_$v.log
done
