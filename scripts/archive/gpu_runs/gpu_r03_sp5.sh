#!/bin/bash
# Round 3: fused pass vs scan pass (PBS_FUSED_MIN_AVG above the average) at 128 and 256 KiB,
# VM image and random, same process.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r03_sp5}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step vm128k 400 env DIAG_CONFIGS="PBS_FUSED_MIN_AVG=131072;PBS_FUSED_MIN_AVG=524288" python scripts/pass_diag.py 64 vmimage 131072 8 || exit 1
step rnd128k 400 env DIAG_CONFIGS="PBS_FUSED_MIN_AVG=131072;PBS_FUSED_MIN_AVG=524288" python scripts/pass_diag.py 64 random 131072 8 || exit 1
step vm256k 400 env DIAG_CONFIGS="PBS_FUSED_MIN_AVG=131072;PBS_FUSED_MIN_AVG=524288" python scripts/pass_diag.py 64 vmimage 262144 8 || exit 1
step rnd256k 400 env DIAG_CONFIGS="PBS_FUSED_MIN_AVG=131072;PBS_FUSED_MIN_AVG=524288" python scripts/pass_diag.py 64 random 262144 8 || exit 1
echo done
