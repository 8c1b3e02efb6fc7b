#!/bin/bash
# fused pass, large averages: round-4 resolver (scripts/ab_libs/libpbschunk_h4.so) vs the tree's build, alternating
set -o pipefail
mkdir -p gpurun_out/fo
for r in 1 2 3; do
  PBS_LIBPBSCHUNK_AB=scripts/ab_libs/libpbschunk_h4.so timeout -k 10 200 python scripts/scan_pass_split.py --kinds vmimage,random --avgs 524288,1048576,4194304 --steps 5 > gpurun_out/fo/old_$r.log 2>&1 || exit 1
  timeout -k 10 200 python scripts/scan_pass_split.py --kinds vmimage,random --avgs 524288,1048576,4194304 --steps 5 > gpurun_out/fo/new_$r.log 2>&1 || exit 1
done
