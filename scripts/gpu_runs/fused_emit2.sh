#!/bin/bash
# fused pass at small averages (forced from 64 KiB) vs the scan pass, 64 GiB, same box
set -o pipefail
mkdir -p gpurun_out/fe2
timeout -k 10 200 python scripts/scan_pass_split.py --kinds vmimage,random --avgs 65536,131072,262144,4194304 --steps 4 > gpurun_out/fe2/default.log 2>&1 || exit 1
PBS_FUSED_MIN_AVG=65536 PBS_DEBUG_PHASES=1 timeout -k 10 200 python scripts/scan_pass_split.py --kinds vmimage,random --avgs 65536,131072,262144,4194304 --steps 4 > gpurun_out/fe2/fused.log 2>&1 || exit 1
