#!/bin/bash
# more, shorter rounds (PBS_STATIC_QMAX) with / without the pool: 8 GiB and 64 GiB
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=gpurun_out/r02bb; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
C8="PBS_POOL_DIV=0;PBS_STATIC_QMAX=160,PBS_POOL_DIV=0;PBS_STATIC_QMAX=160,PBS_POOL_DIV=8,PBS_POOL_ROUND=4;PBS_STATIC_QMAX=80,PBS_POOL_DIV=8,PBS_POOL_ROUND=4"
step c2 300 env DIAG_CONFIGS="$C8" python scripts/pass_diag.py 8 random 4194304 30 || exit 1
C64="PBS_STATIC_QMAX=319;PBS_STATIC_QMAX=200;PBS_STATIC_QMAX=160"
step c3 400 env DIAG_CONFIGS="$C64" python scripts/pass_diag.py 64 vmimage 4194304 5 || exit 1
echo done
