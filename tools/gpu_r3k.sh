# eager host path: pooled gradient buffers + direct parameter gradients; new GPU tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_grad_pool.py tests/test_gpu_defer.py tests/test_gpu_parity.py > gpurun_out/tests_k.log 2>&1 &&
timeout -k 10 200 python -u bench.py > gpurun_out/bench_k.log 2>&1 &&
timeout -k 10 200 python -u bench.py --param-grads direct > gpurun_out/bench_k_direct.log 2>&1 &&
timeout -k 10 300 python -u tools/host_profile.py --steps 200 > gpurun_out/host_profile_k.txt 2>&1 &&
timeout -k 10 300 python -u tools/host_profile.py --steps 200 --param-grads direct > gpurun_out/host_profile_k_direct.txt 2>&1
