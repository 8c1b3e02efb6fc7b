#!/bin/bash
# fused pass resolver helpers: 4 (scripts/ab_libs/libpbschunk_h4.so) vs the tree's build, averages 64 KiB - 4 MiB forced fused
set -o pipefail
mkdir -p gpurun_out/fh
for r in 1 2; do
  PBS_LIBPBSCHUNK_AB=scripts/ab_libs/libpbschunk_h4.so PBS_FUSED_MIN_AVG=65536 PBS_DEBUG_PHASES=1 timeout -k 10 200 python scripts/scan_pass_split.py --kinds vmimage,random --avgs 65536,131072,262144,4194304 --steps 4 > gpurun_out/fh/h4_$r.log 2>&1 || exit 1
  PBS_FUSED_MIN_AVG=65536 PBS_DEBUG_PHASES=1 timeout -k 10 200 python scripts/scan_pass_split.py --kinds vmimage,random --avgs 65536,131072,262144,4194304 --steps 4 > gpurun_out/fh/new_$r.log 2>&1 || exit 1
done
