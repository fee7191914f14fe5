#!/bin/bash
# round 3 session f: ABI v9 (lindisp / perturb), full GPU suite, C2 bench
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r3f
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_strat_options.py > $O/tests_strat.log 2>&1
rc=$?; echo "strat tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/tests_all.log 2>&1
rc=$?; echo "all tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --cpu-seconds 5 > $O/bench_c2.log 2>&1
echo "bench rc=$?"
