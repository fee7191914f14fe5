#!/bin/bash
# round 4 session f: range-guard recompute folded into the compositing kernels (no k_mlp_fwd_exact node):
# A/B against the previous commit's library, then the tests that exercise the guard and compositing
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4f
mkdir -p $O
step() { # name seconds cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "[$n] rc=$rc"; tail -6 $O/$n.log | cut -c1-1500
  if [ $rc -ge 124 ]; then exit $rc; fi
}
step ab 600 python3 -u tools/ablate.py run r4idx r4guard r4idx r4guard
step tests 900 python3 -u -m pytest tests/test_gpu_range_guard.py tests/test_gpu_loss.py tests/test_gpu_parity.py tests/test_gpu_ray_mask.py tests/test_importance.py tests/test_gpu_imap.py tests/test_gpu_render_img.py -m gpu -q --timeout 300 --timeout-method thread
