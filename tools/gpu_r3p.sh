# iMAP*: W_0 forward on the split kernel (scalar B rows); parity, bench, SQ counters
set -o pipefail
mkdir -p gpurun_out/p
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_imap.py > gpurun_out/p/tests_imap.log 2>&1 &&
timeout -k 10 200 python -u tools/bench_imap.py > gpurun_out/p/bench_imap_h.log 2>&1 &&
bash tools/pmc_imap.sh p > gpurun_out/p/pmc.log 2>&1 &&
python tools/pmc_report.py gpurun_out/pmc_imap_p > gpurun_out/p/pmc_report.txt 2>&1
