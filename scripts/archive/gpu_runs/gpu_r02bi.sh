#!/bin/bash
# DPP prefix sums (tile-end publish, helper gather, chain emit) and readlanes for uniform lanes: GPU tests;
# 64 KiB multi-launch (scan_exact), 256 KiB and 4 MiB fused A/B against the HEAD build
# (scripts/ab/libpbschunk_head.so), alternating processes.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=gpurun_out/r02bi; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || exit 1
for r in 1 2; do
  DIAG_CONFIGS="PBS_FUSED=0" DIAG_LIB=scripts/ab/libpbschunk_head.so step head64k_$r 240 python scripts/pass_diag.py 64 vmimage 65536 5 || exit 1
  DIAG_CONFIGS="PBS_FUSED=0" step new64k_$r 240 python scripts/pass_diag.py 64 vmimage 65536 5 || exit 1
  DIAG_CONFIGS="PBS_FUSED=1" DIAG_LIB=scripts/ab/libpbschunk_head.so step head256k_$r 240 python scripts/pass_diag.py 64 vmimage 262144 8 || exit 1
  DIAG_CONFIGS="PBS_FUSED=1" step new256k_$r 240 python scripts/pass_diag.py 64 vmimage 262144 8 || exit 1
  DIAG_CONFIGS="PBS_FUSED=1" DIAG_LIB=scripts/ab/libpbschunk_head.so step head4m_$r 240 python scripts/pass_diag.py 64 vmimage 4194304 8 || exit 1
  DIAG_CONFIGS="PBS_FUSED=1" step new4m_$r 240 python scripts/pass_diag.py 64 vmimage 4194304 8 || exit 1
done
echo done
