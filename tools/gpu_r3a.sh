#!/bin/bash
# round 3, first GPU session: new config parity tests, sparse tests, bench --gpus 2 (gloo)
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r3a
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_configs.py tests/test_gpu_sparse.py > $O/tests.log 2>&1
rc=$?
echo "tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --gpus 2 --backend gloo --steps 10 --warmup 3 --cpu-seconds 0 > $O/bench_gloo2.log 2>&1
rc=$?
echo "bench gloo2 rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --cpu-seconds 5 > $O/bench_c2.log 2>&1
echo "bench c2 rc=$?"
