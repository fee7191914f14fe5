#!/bin/bash
# round 3 session ac: fused forward at 12 waves (one-round-trip gathers), k_mlp_dx channels-last
# instantiation; whole GPU suite, smoke, bench, render_img, Mesher
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r3ac
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/tests_all.log 2>&1
rc=$?; echo "all tests rc=$rc"; tail -2 $O/tests_all.log; grep FAILED $O/tests_all.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc=$?"
timeout -k 10 300 python -u bench.py > $O/bench_c2.log 2>&1; echo "bench rc=$?"
grep -o '"ms_per_step": [0-9.]*\|"eager_direct_ms_per_step": [0-9.]*\|"kernels_ms": {[^}]*}' $O/bench_c2.log
timeout -k 10 300 python3 tools/bench_render_img.py > $O/render_img.log 2>&1; echo "render_img rc=$?"; tail -1 $O/render_img.log
timeout -k 10 300 python3 tools/bench_mesher_query.py > $O/mesher_query.log 2>&1; echo "mesher rc=$?"; tail -1 $O/mesher_query.log
