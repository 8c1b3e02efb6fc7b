#!/bin/bash
# fused pass: main resolver wave alone on its SIMD (PBS_FUSED_MAIN_ALONE=1) vs sharing it with a helper, forced fused from 64 KiB
set -o pipefail
mkdir -p gpurun_out/fa
for r in 1 2; do
  for m in 0 1; do
    PBS_FUSED_MAIN_ALONE=$m PBS_FUSED_MIN_AVG=65536 PBS_DEBUG_PHASES=1 timeout -k 10 200 python scripts/scan_pass_split.py --kinds vmimage,random --avgs 65536,131072,262144,4194304 --steps 4 > gpurun_out/fa/m${m}_$r.log 2>&1 || exit 1
  done
done
