#!/bin/bash
# TCC atomic / write request counters of the library kernels (one pass).
#   tools/pmc_atomic.sh <tag> [bench args...]
tag="$1"; shift
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
out="$ROOT/gpurun_out/pmcA_$tag"
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 120 rocprofv3 --pmc TCC_EA0_ATOMIC_sum TCC_EA0_WRREQ_sum --kernel-include-regex "nc::" --output-format csv \
    -d "$out/p1" -o run -- python3 "$ROOT/bench.py" --eager --cpu-seconds 0 "$@" > "$out/p1.log" 2>&1
