#!/bin/bash
# fused pass with the entry table (main wave: two readlanes a vector) and helper-written cuts: parity subset, then
# the scan pass (committed policy: PBS_FUSED_MIN_AVG default) vs the fused pass forced from 64 KiB, and the large averages
set -o pipefail
mkdir -p gpurun_out/ff
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "fused or scan_pass or chunker1 or feed or full_size" > gpurun_out/ff/tests.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 200 python scripts/scan_pass_split.py --kinds vmimage,random --avgs 65536,131072,262144,1048576,4194304 --steps 5 > gpurun_out/ff/default_$r.log 2>&1 || exit 1
  PBS_FUSED_MIN_AVG=65536 PBS_DEBUG_PHASES=1 timeout -k 10 200 python scripts/scan_pass_split.py --kinds vmimage,random --avgs 65536,131072,262144 --steps 5 > gpurun_out/ff/fused_$r.log 2>&1 || exit 1
done
