# iMAP* split-f16 layer GEMMs: parity, A/B against the f32 kernel, kernel stats
set -o pipefail
mkdir -p gpurun_out/l
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_imap.py > gpurun_out/l/tests_imap.log 2>&1 &&
timeout -k 10 200 python -u tools/bench_imap.py > gpurun_out/l/bench_imap_h.log 2>&1 &&
NC_IMAP_F32=1 timeout -k 10 200 python -u tools/bench_imap.py > gpurun_out/l/bench_imap_f32.log 2>&1 &&
timeout -k 10 200 python -u tools/bench_imap.py --mode tracker > gpurun_out/l/bench_imap_h_tracker.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/l/prof -o imap -- python3 tools/bench_imap.py --steps 5 > gpurun_out/l/prof.log 2>&1
