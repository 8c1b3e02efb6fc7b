#!/bin/bash
# static order with / without workgroup 0's scanner waves (the resolver shares CU 0)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=gpurun_out/r02as; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step fused_tests 600 python -u -m pytest tests/test_gpu_parity.py -k "fused or golden or split" -x -v --timeout 300 --timeout-method thread || exit 1
C="PBS_SCAN_DYN=1;PBS_SCAN_DYN=0,PBS_WG0_SCAN=1;PBS_SCAN_DYN=0,PBS_WG0_SCAN=0"
step c5 400 env PBS_FUSED=1 DIAG_CONFIGS="$C" python scripts/pass_diag.py 64 vmimage 262144 5 || exit 1
step c3 400 env DIAG_CONFIGS="$C" python scripts/pass_diag.py 64 vmimage 4194304 5 || exit 1
step c2 300 env PBS_FUSED=1 DIAG_CONFIGS="$C" python scripts/pass_diag.py 8 random 4194304 30 || exit 1
step c5_8 300 env PBS_FUSED=1 DIAG_CONFIGS="PBS_FUSED=0;PBS_SCAN_DYN=0,PBS_WG0_SCAN=1,PBS_FUSED=1;PBS_SCAN_DYN=0,PBS_WG0_SCAN=0,PBS_FUSED=1" python scripts/pass_diag.py 8 vmimage 262144 30 || exit 1
echo done
