#!/bin/bash
# round 4 session r: where the NC_DETERMINISTIC step's time goes (bench line + rocprofv3 stats)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4r
mkdir -p $O
step() { # name seconds cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "[$n] rc=$rc"; tail -2 $O/$n.log | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
}
NC_DETERMINISTIC=1 step bench 300 python3 -u bench.py --steps 50 --warmup 5 --cpu-seconds 0
NC_DETERMINISTIC=1 step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 "$f" | head -20
