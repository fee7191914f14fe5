#!/bin/bash
# Round-3 (re-entry) evidence for the NICE path on the current kernels: whole GPU suite + smoke,
# rocprofv3 stats + HBM traffic of the headline bench, SQ counters, config lines, forward-only
# reuse, headline bench line.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/al
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/tests_all.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
bash tools/prof_session.sh al > $O/prof_session.log 2>&1 &&
bash tools/pmc_session.sh al > $O/pmc_session.log 2>&1 &&
python3 tools/pmc_report.py gpurun_out/pmc_al > $O/pmc_report.txt 2>&1 &&
bash tools/configs_session.sh al > $O/configs.log 2>&1 &&
timeout -k 10 300 python3 tools/bench_render_img.py > $O/render_img.log 2>&1 &&
timeout -k 10 300 python3 tools/bench_mesher_query.py > $O/mesher_query.log 2>&1 &&
timeout -k 10 300 python3 bench.py > $O/bench_c2.log 2>&1
