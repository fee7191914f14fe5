#!/bin/bash
# Bench lines for the BASELINE.json configs beyond the headline (1 GPU each):
# C1 Replica room0 200 rays, stage middle, no render depth (S = 32), C3 ScanNet 5000 rays (+ coarse mapper pass), C4 Apartment 625-ray shard, C5 synthetic
# 200M-voxel grids with sparse rows (2048 and 16384 rays), tracker mode at C2.
#   tools/configs_session.sh <tag>
tag="$1"
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
out="$ROOT/gpurun_out/cfg_$tag"
mkdir -p "$out"
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { name="$1"; shift; echo "=== $name"; timeout -k 10 240 python3 "$ROOT/bench.py" "$@" > "$out/$name.log" 2>&1; rc=$?; tail -c 300 "$out/$name.log"; echo; return $rc; }
run c1 --stage middle --rays 200 --render-depth none --steps 30 --cpu-seconds 10 &&
run c3 --scene scannet_scene0000 --rays 5000 --steps 20 --cpu-seconds 0 &&
run c3coarse --scene scannet_scene0000 --rays 5000 --stage coarse --steps 20 --cpu-seconds 0 &&
run c4 --scene apartment --rays 625 --steps 20 --cpu-seconds 0 &&
run c5 --scene synthetic_c5 --rays 2048 --steps 10 --warmup 2 --cpu-seconds 0 &&
run c5_16k --scene synthetic_c5 --rays 16384 --steps 10 --warmup 2 --cpu-seconds 0 &&
run tracker --mode tracker --steps 30 --cpu-seconds 0 &&
run fix_fine --fix-fine --steps 30 --cpu-seconds 0 &&
run iteration --iteration --steps 30 --cpu-seconds 0
