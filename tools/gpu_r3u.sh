#!/bin/bash
# round 3 session u (re-entry): full GPU suite + smoke + bench on the restored tree
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r3u
mkdir -p $O
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/tests_all.log 2>&1
rc=$?; echo "all tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py > $O/bench_c2.log 2>&1
rc=$?; echo "bench rc=$rc"
exit $rc
