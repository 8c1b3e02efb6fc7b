#!/bin/bash
# Fused main wave: LDS cut buffer + 8 resolver vectors in flight (ring walked in place, nf|xl packed):
# GPU tests; 64 KiB and 128 KiB averages fused vs multi-launch; 4 MiB and 256 KiB A/B
# against the HEAD build (scripts/ab/libpbschunk_head.so), same box.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=gpurun_out/r02bf; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || exit 1
DIAG_CONFIGS="PBS_FUSED=0;PBS_FUSED_MIN_AVG=65536,PBS_SCAN_DYN=1,PBS_DEBUG_PHASES=1;PBS_FUSED_MIN_AVG=65536,PBS_SCAN_DYN=0,PBS_DEBUG_PHASES=1" step a64k 300 python scripts/pass_diag.py 64 vmimage 65536 5 || exit 1
DIAG_CONFIGS="PBS_FUSED=0;PBS_SCAN_DYN=1;PBS_SCAN_DYN=0" step a128k 300 python scripts/pass_diag.py 64 vmimage 131072 5 || exit 1
for r in 1 2; do
  DIAG_CONFIGS="PBS_FUSED=1" DIAG_LIB=scripts/ab/libpbschunk_head.so step head4m_$r 240 python scripts/pass_diag.py 64 vmimage 4194304 10 || exit 1
  DIAG_CONFIGS="PBS_FUSED=1" step new4m_$r 240 python scripts/pass_diag.py 64 vmimage 4194304 10 || exit 1
done
DIAG_CONFIGS="PBS_FUSED=1" DIAG_LIB=scripts/ab/libpbschunk_head.so step head256k 240 python scripts/pass_diag.py 64 vmimage 262144 10 || exit 1
DIAG_CONFIGS="PBS_FUSED=1" step new256k 240 python scripts/pass_diag.py 64 vmimage 262144 10 || exit 1
DIAG_CONFIGS="PBS_FUSED=0;PBS_FUSED_MIN_AVG=65536" step r8_64k 240 python scripts/pass_diag.py 8 random 65536 10 || exit 1
echo done
