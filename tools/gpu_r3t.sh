# iMAP*: split-f16 forward + dX GEMMs (transposed weights), f32 dW; parity + A/B
set -o pipefail
mkdir -p gpurun_out/t
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_imap.py > gpurun_out/t/tests_imap.log 2>&1 &&
timeout -k 10 200 python -u tools/bench_imap.py > gpurun_out/t/bench_imap_h.log 2>&1 &&
NC_IMAP_F32=1 timeout -k 10 200 python -u tools/bench_imap.py > gpurun_out/t/bench_imap_f32.log 2>&1 &&
timeout -k 10 200 python -u tools/bench_imap.py --mode tracker > gpurun_out/t/bench_imap_h_tracker.log 2>&1 &&
NC_IMAP_F32=1 timeout -k 10 200 python -u tools/bench_imap.py --mode tracker > gpurun_out/t/bench_imap_f32_tracker.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/t/prof -o imap -- python3 tools/bench_imap.py --steps 5 > gpurun_out/t/prof.log 2>&1
