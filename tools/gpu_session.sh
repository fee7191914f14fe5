#!/bin/bash
# Run a sequence of GPU steps on the gpurun box, each under its own time limit.
# Stops at the first crash / fault / timeout (exit 124,137,134,139 or >128);
# ordinary failures (pytest exit 1) are reported and the next step runs.
# usage: tools/gpu_session.sh "name:seconds:command" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== [$name] (limit ${secs}s) $cmd"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc in $(( $(date +%s) - start ))s"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ] || [ $rc -gt 128 ]; then
    echo "=== stopping: step $name ended abnormally (rc=$rc)"
    exit $rc
  fi
done
exit 0
