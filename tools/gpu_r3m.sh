# split-f16 iMAP GEMM at 2 waves/SIMD: A/B kernel stats
set -o pipefail
mkdir -p gpurun_out/m
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/m/prof -o imap -- python3 tools/bench_imap.py --steps 5 > gpurun_out/m/prof.log 2>&1 &&
timeout -k 10 200 python -u tools/bench_imap.py > gpurun_out/m/bench_imap_h.log 2>&1
