#!/bin/bash
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r3z
mkdir -p $O
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_loss.py tests/test_gpu_determinism.py tests/test_gpu_defer.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; grep FAILED $O/tests.log | head
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 python -u bench.py --cpu-seconds 0 > $O/bench.log 2>&1; echo "bench rc=$?"
grep -o '"ms_per_step": [0-9.]*\|"eager_direct_ms_per_step": [0-9.]*\|"kernels_ms": {[^}]*}' $O/bench.log
