#!/bin/bash
# round 3 session aa: k_mlp_fwd stores each tile's records after the next tile's gathers
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r3aa
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/tests_all.log 2>&1
rc=$?; echo "all tests rc=$rc"; tail -2 $O/tests_all.log; grep FAILED $O/tests_all.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for v in 1 2; do
  timeout -k 10 120 python -u bench.py --cpu-seconds 0 > $O/bench_$v.log 2>&1
  rc=$?; echo "bench rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
  grep -o '"ms_per_step": [0-9.]*\|"kernels_ms": {[^}]*}' $O/bench_$v.log
done
timeout -k 10 300 python3 tools/bench_render_img.py > $O/render_img.log 2>&1; echo "render_img rc=$?"; tail -3 $O/render_img.log
timeout -k 10 300 python3 tools/bench_mesher_query.py > $O/mesher_query.log 2>&1; echo "mesher rc=$?"; tail -3 $O/mesher_query.log
