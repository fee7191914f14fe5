#!/bin/bash
# round 3 session aj: xor 16 / 32 via v_permlane16/32_swap (sum_groups, scatter face shift, wave sums)
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r3ak
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/tests_all.log 2>&1
rc=$?; echo "all tests rc=$rc"; tail -2 $O/tests_all.log; grep FAILED $O/tests_all.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 500 python -u tools/ablate.py run prev5 cur prev5 cur > $O/ablate.log 2>&1; echo "ablate rc=$?"; cat $O/ablate.log
