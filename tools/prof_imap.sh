#!/bin/bash
# rocprofv3 kernel trace + stats of one tools/bench_imap.py run (iMAP* Mapper iteration).
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
out="$ROOT/gpurun_out/prof_imap"
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/stats" -o run -- \
    python3 "$ROOT/tools/bench_imap.py" --steps 10 > "$out/stats.log" 2>&1
rc=$?
tail -n 3 "$out/stats.log"
exit $rc
