#!/bin/bash
# round 4 session a: init-std parity (golden + exact C2 bench workload), then the bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4a
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_initstd.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests_initstd.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 $O/tests_initstd.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > $O/bench_c2.log 2>&1
echo "bench rc=$?"; tail -c 600 $O/bench_c2.log
