#!/bin/bash
# round 3 session g: Fourier-B gradient moved into k_mlp_dx (record -384 B/pt): parity + A/B timing
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r3g
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_defer.py tests/test_gpu_determinism.py tests/test_gpu_loss.py \
  tests/test_gpu_sparse.py tests/test_gpu_configs.py tests/test_strat_options.py tests/test_gpu_adam.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u tools/ablate.py run prev base prev base > $O/ab.log 2>&1
echo "ab rc=$?"
