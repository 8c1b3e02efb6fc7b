#!/bin/bash
# Round 3: where the fused kernel's extra time at small averages goes -- the same stream
# through the fused pass (resolver waves) and the scan pass (no resolver; forced with
# PBS_FUSED_MIN_AVG above the average), same process, 64 GiB VM image at 256 KiB and 4 MiB.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r03_sp4}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step vm256k 400 env DIAG_CONFIGS="PBS_FUSED_MIN_AVG=131072;PBS_FUSED_MIN_AVG=524288" python scripts/pass_diag.py 64 vmimage 262144 8 || exit 1
step vm4m 400 env DIAG_CONFIGS="PBS_FUSED_MIN_AVG=131072;PBS_FUSED_MIN_AVG=8388608" python scripts/pass_diag.py 64 vmimage 4194304 8 || exit 1
echo done
