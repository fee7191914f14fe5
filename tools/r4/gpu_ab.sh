#!/bin/bash
# round 4 session ab: k_det_join neighbour keys together, pieces 4 ahead, row descriptors
# determinism tests, then A/B of the NC_DETERMINISTIC step (head / current / no XCD order)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4ab
mkdir -p $O
step() { # name seconds cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "[$n] rc=$rc"; tail -5 $O/$n.log | cut -c1-400
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step det_tests 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_determinism.py
NC_DETERMINISTIC=1 step ab 400 python3 -u tools/ablate.py run det_aa cur det_aa cur
NC_DETERMINISTIC=1 step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0
