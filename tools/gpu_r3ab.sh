#!/bin/bash
# round 3 session ab: fused forward gathers every corner of a tile in one round trip
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r3ab
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/tests_all.log 2>&1
rc=$?; echo "all tests rc=$rc"; tail -2 $O/tests_all.log; grep FAILED $O/tests_all.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u tools/ablate.py run cur fwd_b2 cur fwd_b2 > $O/ablate.log 2>&1; echo "ablate rc=$?"; cat $O/ablate.log
timeout -k 10 300 python3 tools/bench_render_img.py > $O/render_img.log 2>&1; echo "render_img rc=$?"; tail -1 $O/render_img.log
timeout -k 10 300 python3 tools/bench_mesher_query.py > $O/mesher_query.log 2>&1; echo "mesher rc=$?"; tail -1 $O/mesher_query.log
