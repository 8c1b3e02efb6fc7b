#!/bin/bash
# HEAD build (static + short last round) vs working tree (static + pool), same box; anchor = dynamic order
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=gpurun_out/r02aq; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step head_c3 300 env DIAG_LIB=scripts/ab/libpbschunk_head.so DIAG_CONFIGS="PBS_SCAN_DYN=1;PBS_SCAN_DYN=0" python scripts/pass_diag.py 64 vmimage 4194304 5 || exit 1
step cur_c3 300 env DIAG_CONFIGS="PBS_SCAN_DYN=1;PBS_SCAN_DYN=0,PBS_POOL_PCT=0;PBS_SCAN_DYN=0,PBS_POOL_PCT=25" python scripts/pass_diag.py 64 vmimage 4194304 5 || exit 1
step head_c2 300 env PBS_FUSED=1 DIAG_LIB=scripts/ab/libpbschunk_head.so DIAG_CONFIGS="PBS_SCAN_DYN=1;PBS_SCAN_DYN=0" python scripts/pass_diag.py 8 random 4194304 30 || exit 1
step cur_c2 300 env PBS_FUSED=1 DIAG_CONFIGS="PBS_SCAN_DYN=1;PBS_SCAN_DYN=0,PBS_POOL_PCT=0;PBS_SCAN_DYN=0,PBS_POOL_PCT=25" python scripts/pass_diag.py 8 random 4194304 30 || exit 1
echo done
