#!/bin/bash
# zero-fill with non-temporal stores (NC_ZERO_NT) A/B
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/ao
mkdir -p $O
timeout -k 10 500 python -u tools/ablate.py run cur zero_nt cur zero_nt cur zero_nt > $O/ab_zero_nt.log 2>&1
