set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/host_profile.py --steps 200 > gpurun_out/host_profile_j.txt 2>&1 &&
timeout -k 10 200 python -u tools/host_micro.py > gpurun_out/host_micro_j.txt 2>&1 &&
timeout -k 10 200 python -u bench.py > gpurun_out/bench_j.log 2>&1
