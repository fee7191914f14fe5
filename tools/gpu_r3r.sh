set -o pipefail
mkdir -p gpurun_out/q
timeout -k 10 300 python3 tools/bench_render_img.py > gpurun_out/q/render_img.log 2>&1 &&
timeout -k 10 300 python3 tools/bench_mesher_query.py > gpurun_out/q/mesher_query.log 2>&1 &&
timeout -k 10 300 python3 bench.py > gpurun_out/q/bench_c2.log 2>&1
