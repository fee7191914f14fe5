#!/bin/bash
# round 3 session b: range guard, iMAP* gate, C5 window test, full GPU suite, C2 bench
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r3b
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_range_guard.py tests/test_gpu_imap.py "tests/test_gpu_configs.py::test_c5_256_rays_match_oracle_on_grid_windows" > $O/tests_new.log 2>&1
rc=$?; echo "new tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/tests_all.log 2>&1
rc=$?; echo "all tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --cpu-seconds 5 > $O/bench_c2.log 2>&1
echo "bench rc=$?"
