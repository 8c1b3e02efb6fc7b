#!/bin/bash
# Round 3: tile order at 128 KiB averages (fused pass), static vs dynamic, same process
# (pass_diag alternates the settings), 64 GiB VM image and 64 GiB random.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r03_s128}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step vm128k 400 env DIAG_CONFIGS="PBS_SCAN_DYN=0;PBS_SCAN_DYN=1" python scripts/pass_diag.py 64 vmimage 131072 8 || exit 1
step rnd128k 400 env DIAG_CONFIGS="PBS_SCAN_DYN=0;PBS_SCAN_DYN=1" python scripts/pass_diag.py 64 random 131072 8 || exit 1
echo done
