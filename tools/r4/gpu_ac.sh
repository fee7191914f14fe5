#!/bin/bash
# round 4 session ac: k_det_join (neighbour keys together, pieces 4 ahead, row descriptors)
# and the per-ray kernels' loads made unconditional (k_ray_setup inputs and batch max, sample_state,
# in_bound, ray_ok, the fused loss targets)
# then same-box A/B of the default step and of the NC_DETERMINISTIC step
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4ac
mkdir -p $O
step() { # name seconds cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "[$n] rc=$rc"; tail -6 $O/$n.log | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step ab 400 python3 -u tools/ablate.py run cur rays_hoist cur rays_hoist cur rays_hoist
NC_DETERMINISTIC=1 step ab_det 400 python3 -u tools/ablate.py run det_aa cur rays_hoist det_aa cur rays_hoist
NC_DETERMINISTIC=1 step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0
