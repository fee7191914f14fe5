#!/bin/bash
# round 3 session d: exact-gate launch change (range guard tests + bench), host profile of the eager step
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r3d
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_range_guard.py tests/test_gpu_parity.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --cpu-seconds 0 > $O/bench_c2.log 2>&1
rc=$?; echo "bench rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/host_profile.py --steps 100 > $O/host_profile.txt 2>&1
echo "host rc=$?"
