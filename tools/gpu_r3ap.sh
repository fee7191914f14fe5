#!/bin/bash
# whole Tracker iteration on the drop-ins (sampling + bbox filter + render + loss + backward to the camera + Adam)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/ap
mkdir -p $O
timeout -k 10 300 python3 -u tools/bench_tracker_iteration.py > $O/tracker_iteration.log 2>&1 &&
cd /tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ap/prof -o trk -- python3 tools/bench_tracker_iteration.py --iters 50 > $O/prof.log 2>&1
