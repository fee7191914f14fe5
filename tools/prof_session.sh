#!/bin/bash
# rocprofv3 evidence for profiles/: kernel trace + stats of the bench command, then
# HBM traffic counters in separate passes (FETCH_SIZE and WRITE_SIZE cannot share
# one pass on gfx950).  Run from the repo root on the GPU box.
#   tools/prof_session.sh <tag> [bench args...]
tag="$1"; shift
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
out="$ROOT/gpurun_out/prof_$tag"
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() {  # name seconds args...
  local name="$1" secs="$2"; shift 2
  echo "=== $name"
  timeout -k 10 "$secs" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 3 "$out/$name.log"
  return $rc
}
run stats 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/stats" -o run -- \
    python3 "$ROOT/bench.py" "$@" --cpu-seconds 0 &&
run fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o run -- \
    python3 "$ROOT/bench.py" "$@" --cpu-seconds 0 &&
run write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o run -- \
    python3 "$ROOT/bench.py" "$@" --cpu-seconds 0 &&
run atomic 300 rocprofv3 --pmc TCC_EA0_ATOMIC_sum --output-format csv -d "$out/atomic" -o run -- \
    python3 "$ROOT/bench.py" "$@" --cpu-seconds 0 &&
python3 "$ROOT/tools/pmc_traffic.py" --atomic "$out/atomic" "$out/fetch" "$out/write" "$out/hbm_traffic.json" "$@"
