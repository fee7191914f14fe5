#!/bin/bash
# round 3 session h: launch cost, host micro-timings, k_mlp_dw shape A/B
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r3h
mkdir -p $O
timeout -k 10 120 ./tools/launch_cost_bin > $O/launch_cost.txt 2>&1
echo "launch rc=$?"
timeout -k 10 300 python -u tools/host_micro.py > $O/host_micro.txt 2>&1
echo "micro rc=$?"
timeout -k 10 900 python -u tools/ablate.py run base dw_npts48 dw768_32 dw_npts16 base dw_npts48 dw768_32 dw_npts16 > $O/ab.log 2>&1
echo "ab rc=$?"
