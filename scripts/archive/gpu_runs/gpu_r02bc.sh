#!/bin/bash
# 64 KiB averages through the fused pass (four helpers now) vs the multi-launch path
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=gpurun_out/r02bc; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
C="PBS_FUSED=0;PBS_FUSED_MIN_AVG=65536,PBS_SCAN_DYN=1;PBS_FUSED_MIN_AVG=65536,PBS_SCAN_DYN=0;PBS_FUSED_MIN_AVG=65536,PBS_SCAN_DYN=0,PBS_POOL_DIV=0"
step a64k 500 env PBS_DEBUG_PHASES=1 DIAG_CONFIGS="$C" python scripts/pass_diag.py 64 vmimage 65536 3 || exit 1
step a128 400 env DIAG_CONFIGS="PBS_FUSED=0;PBS_SCAN_DYN=1" python scripts/pass_diag.py 64 vmimage 131072 4 || exit 1
echo done
