#!/bin/bash
# whole Tracker iteration: eager vs one hipGraph per iteration
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/aq
mkdir -p $O
timeout -k 10 300 python3 -u tools/bench_tracker_iteration.py --graph > $O/tracker_iteration_graph.log 2>&1
