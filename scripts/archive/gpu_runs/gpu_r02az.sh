#!/bin/bash
# pool size sweep: short round of k/8 round drawn as d x smaller tiles
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=gpurun_out/r02az; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
C="PBS_POOL_DIV=0,PBS_POOL_ROUND=1;PBS_POOL_DIV=4,PBS_POOL_ROUND=1;PBS_POOL_DIV=4,PBS_POOL_ROUND=2;PBS_POOL_DIV=8,PBS_POOL_ROUND=4;PBS_POOL_DIV=8,PBS_POOL_ROUND=8;PBS_POOL_DIV=16,PBS_POOL_ROUND=8"
step c3 500 env DIAG_CONFIGS="$C" python scripts/pass_diag.py 64 vmimage 4194304 5 || exit 1
step r64 500 env DIAG_CONFIGS="$C" python scripts/pass_diag.py 64 random 4194304 4 || exit 1
step c2 300 env DIAG_CONFIGS="$C" python scripts/pass_diag.py 8 random 4194304 30 || exit 1
echo done
