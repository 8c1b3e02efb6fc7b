#!/bin/bash
# no scratch spills: HEAD build vs working tree (pool variants), same box
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=gpurun_out/r02ar; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step fused_tests 600 python -u -m pytest tests/test_gpu_parity.py -k "fused or golden or split" -x -v --timeout 300 --timeout-method thread || exit 1
step head_c3 300 env DIAG_LIB=scripts/ab/libpbschunk_head.so DIAG_CONFIGS="PBS_SCAN_DYN=1;PBS_SCAN_DYN=0" python scripts/pass_diag.py 64 vmimage 4194304 5 || exit 1
step cur_c3 400 env DIAG_CONFIGS="PBS_SCAN_DYN=1;PBS_SCAN_DYN=0,PBS_POOL_PCT=0;PBS_SCAN_DYN=0,PBS_POOL_PCT=25,PBS_POOL_DIV=4;PBS_SCAN_DYN=0,PBS_POOL_PCT=25,PBS_POOL_DIV=8;PBS_SCAN_DYN=0,PBS_POOL_PCT=12,PBS_POOL_DIV=4" python scripts/pass_diag.py 64 vmimage 4194304 5 || exit 1
step head_c2 300 env PBS_FUSED=1 DIAG_LIB=scripts/ab/libpbschunk_head.so DIAG_CONFIGS="PBS_SCAN_DYN=1;PBS_SCAN_DYN=0" python scripts/pass_diag.py 8 random 4194304 30 || exit 1
step cur_c2 300 env PBS_FUSED=1 DIAG_CONFIGS="PBS_SCAN_DYN=1;PBS_SCAN_DYN=0,PBS_POOL_PCT=0;PBS_SCAN_DYN=0,PBS_POOL_PCT=25,PBS_POOL_DIV=4;PBS_SCAN_DYN=0,PBS_POOL_PCT=25,PBS_POOL_DIV=8;PBS_SCAN_DYN=0,PBS_POOL_PCT=12,PBS_POOL_DIV=4" python scripts/pass_diag.py 8 random 4194304 30 || exit 1
step cur_c5 400 env PBS_FUSED=1 DIAG_CONFIGS="PBS_SCAN_DYN=1;PBS_SCAN_DYN=0,PBS_POOL_PCT=25,PBS_POOL_DIV=4;PBS_SCAN_DYN=0,PBS_POOL_PCT=25,PBS_POOL_DIV=8" python scripts/pass_diag.py 64 vmimage 262144 5 || exit 1
echo done
