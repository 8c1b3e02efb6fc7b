#!/bin/bash
# scan_exact_kernel with 4 item windows in flight per wave: GPU tests, then the 64 KiB
# multi-launch pass A/B against the HEAD build (scripts/ab/libpbschunk_head.so), same box.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=gpurun_out/r02bd; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || exit 1
for r in 1 2; do
  DIAG_CONFIGS="PBS_FUSED=0" DIAG_LIB=scripts/ab/libpbschunk_head.so step ab_head_$r 240 python scripts/pass_diag.py 64 vmimage 65536 10 || exit 1
  DIAG_CONFIGS="PBS_FUSED=0" step ab_new_$r 240 python scripts/pass_diag.py 64 vmimage 65536 10 || exit 1
done
DIAG_CONFIGS="PBS_FUSED=0" step ab_new_random8 240 python scripts/pass_diag.py 8 random 65536 10 || exit 1
DIAG_CONFIGS="PBS_FUSED=0" DIAG_LIB=scripts/ab/libpbschunk_head.so step ab_head_random8 240 python scripts/pass_diag.py 8 random 65536 10 || exit 1

# where the fused pass loses at 64 KiB: resolver last record ready vs done (stderr)
DIAG_CONFIGS="PBS_FUSED_MIN_AVG=65536,PBS_SCAN_DYN=1,PBS_DEBUG_PHASES=1" step fused64k_phases 240 python scripts/pass_diag.py 64 vmimage 65536 3 || exit 1
echo done
