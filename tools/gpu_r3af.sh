#!/bin/bash
# round 3 session af: Fourier-B weight gradient in k_mlp_dx on the MFMA (was DPP row sums)
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r3af
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/tests_all.log 2>&1
rc=$?; echo "all tests rc=$rc"; tail -2 $O/tests_all.log; grep FAILED $O/tests_all.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc=$?"; tail -1 $O/smoke.log
timeout -k 10 500 python -u tools/ablate.py run prevb cur prevb cur > $O/ablate.log 2>&1; echo "ablate rc=$?"; cat $O/ablate.log
