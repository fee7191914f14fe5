# Final round-3 evidence for the NICE path (kernels final): rocprofv3 stats + HBM traffic
# of the headline bench, SQ counters, config lines, forward-only reuse, headline bench line.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out/q
bash tools/prof_session.sh final > gpurun_out/q/prof_session.log 2>&1 &&
bash tools/pmc_session.sh final > gpurun_out/q/pmc_session.log 2>&1 &&
python3 tools/pmc_report.py gpurun_out/pmc_final > gpurun_out/q/pmc_report.txt 2>&1 &&
bash tools/configs_session.sh final > gpurun_out/q/configs.log 2>&1 &&
timeout -k 10 300 python3 tools/bench_render_img.py > gpurun_out/q/render_img.log 2>&1 &&
timeout -k 10 300 python3 tools/bench_mesher_query.py > gpurun_out/q/mesher_query.log 2>&1 &&
timeout -k 10 300 python3 bench.py > gpurun_out/q/bench_c2.log 2>&1
