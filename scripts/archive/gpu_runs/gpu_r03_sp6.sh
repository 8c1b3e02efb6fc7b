#!/bin/bash
# Round 3: fused pass vs scan pass at 128 KiB on 8 GiB batches (VM image, random), same process.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r03_sp6}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step vm128k_8g 400 env DIAG_CONFIGS="PBS_FUSED_MIN_AVG=131072,PBS_SCAN_PASS=0;PBS_FUSED_MIN_AVG=524288" python scripts/pass_diag.py 8 vmimage 131072 30 || exit 1
step rnd128k_8g 400 env DIAG_CONFIGS="PBS_FUSED_MIN_AVG=131072,PBS_SCAN_PASS=0;PBS_FUSED_MIN_AVG=524288" python scripts/pass_diag.py 8 random 131072 30 || exit 1
step vm128k_16g 400 env DIAG_CONFIGS="PBS_FUSED_MIN_AVG=131072,PBS_SCAN_PASS=0;PBS_FUSED_MIN_AVG=524288" python scripts/pass_diag.py 16 vmimage 131072 16 || exit 1
step tests_parity 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread || exit 1
echo done
