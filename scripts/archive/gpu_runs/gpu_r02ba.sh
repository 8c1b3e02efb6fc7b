#!/bin/bash
# static order + pool at small averages (64 GiB) vs the dynamic order
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=gpurun_out/r02ba; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
C="PBS_SCAN_DYN=1;PBS_SCAN_DYN=0;PBS_SCAN_DYN=0,PBS_POOL_ROUND=8,PBS_POOL_DIV=8"
step c5 400 env DIAG_CONFIGS="$C" python scripts/pass_diag.py 64 vmimage 262144 5 || exit 1
step a128 400 env DIAG_CONFIGS="$C" python scripts/pass_diag.py 64 vmimage 131072 5 || exit 1
step a512 400 env DIAG_CONFIGS="$C" python scripts/pass_diag.py 64 vmimage 524288 5 || exit 1
echo done
