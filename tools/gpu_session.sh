#!/bin/bash
# The one runner for GPU sessions on the gpurun box: a sequence of steps, each under its
# own time limit, logs under gpurun_out/<tag>/<step>.log.
# Stops at the first crash / fault / timeout (exit 124, 137, 134, 139 or > 128), and at an
# ordinary failure too when GS_STRICT=1; otherwise an ordinary failure (pytest exit 1) is
# reported and the next step runs.
#
#   tools/gpu_session.sh <tag> "name:seconds:command" ...
#
# e.g. the closing evidence of a round:
#   tools/gpu_session.sh r5fin \
#     "tests:900:python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
#     "smoke:300:python3 -u -c 'import __graft_entry__ as g; g.smoke()'" \
#     "bench:300:python3 -u bench.py" \
#     "bench_det:300:NC_DETERMINISTIC=1 python3 -u bench.py" \
#     "prof:900:tools/prof_session.sh r5fin"
# A/B of library variants: build them here first (tools/ablate.py), then one step per
# variant with NICECORE_LIB=<variant.so>.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
tag="$1"; shift
out="gpurun_out/$tag"
mkdir -p "$out"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== [$name] (limit ${secs}s) $cmd"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "$out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc in $(( $(date +%s) - start ))s"
  tail -n 25 "$out/$name.log" | cut -c1-400
  if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ] || [ $rc -gt 128 ]; then
    echo "=== stopping: step $name ended abnormally (rc=$rc)"
    exit $rc
  fi
  if [ $rc -ne 0 ] && [ "${GS_STRICT:-0}" = 1 ]; then
    echo "=== stopping: step $name failed (rc=$rc, GS_STRICT=1)"
    exit $rc
  fi
done
exit 0
