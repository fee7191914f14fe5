#!/bin/bash
# Forward-only benchmarks (render_img frame, Mesher lattice) with rocprofv3 kernel stats.
#   tools/fwd_session.sh <tag>
tag="$1"
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
out="$ROOT/gpurun_out/fwd_$tag"
mkdir -p "$out"
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 200 python3 "$ROOT/tools/bench_render_img.py" --frames 10 > "$out/render_img.log" 2>&1 &&
timeout -k 10 200 python3 "$ROOT/tools/bench_mesher_query.py" --res 256 --reps 3 > "$out/mesher.log" 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/stats_render_img" -o run -- \
    python3 "$ROOT/tools/bench_render_img.py" --frames 3 > "$out/render_img_prof.log" 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/stats_mesher" -o run -- \
    python3 "$ROOT/tools/bench_mesher_query.py" --res 256 --reps 2 > "$out/mesher_prof.log" 2>&1
