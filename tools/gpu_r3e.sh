#!/bin/bash
# round 3 session e: frustum rows, determinism (own radix sort), host micro-timings, det-path kernel stats
cd "$(dirname "$0")/.."
ROOT=$(pwd)
export TMPDIR=/tmp
O=$ROOT/gpurun_out/r3e
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_frustum_rows.py tests/test_gpu_determinism.py tests/test_gpu_range_guard.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/host_micro.py > $O/host_micro.txt 2>&1
rc=$?; echo "host micro rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
cd /tmp && NC_DETERMINISTIC=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/det_stats -o run -- \
   python3 $ROOT/bench.py --cpu-seconds 0 --steps 20 > $O/det_stats.log 2>&1
echo "det stats rc=$?"
