#!/bin/bash
# fused pass with helper-written cuts: parity subset, then 64 GiB split per average (scan pass default vs fused forced)
set -o pipefail
mkdir -p gpurun_out/fe
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "fused or scan_pass or chunker1 or feed" > gpurun_out/fe/tests.log 2>&1 || exit 1
timeout -k 10 200 python scripts/scan_pass_split.py --kinds vmimage,random --avgs 65536,131072,262144,4194304 --steps 4 > gpurun_out/fe/default.log 2>&1 || exit 1
PBS_FUSED_MIN_AVG=65536 PBS_DEBUG_PHASES=1 timeout -k 10 200 python scripts/scan_pass_split.py --kinds vmimage,random --avgs 65536,131072,262144,4194304 --steps 4 > gpurun_out/fe/fused.log 2>&1 || exit 1
