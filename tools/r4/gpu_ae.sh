#!/bin/bash
# round 4 session ae: k_loss's per-ray inputs loaded together (final loop, cached median keys)
# -- the loss / tracker tests, then the tracker-mode C2 step A/B (previous / new library)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4ae
mkdir -p $O
step() { # name seconds cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "[$n] rc=$rc"; tail -3 $O/$n.log | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests 600 python3 -u -m pytest tests/test_gpu_loss.py tests/test_gpu_ray_mask.py -m gpu -x -q --timeout 300 --timeout-method thread
for i in 1 2 3; do
  for v in prevloss newloss; do
    NICECORE_LIB=dbg/abl_$v.so step trk_${v}_$i 300 python3 -u bench.py --mode tracker --steps 50 --warmup 5 --cpu-seconds 0
  done
done
for f in $O/trk_*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f)"; done
