#!/bin/bash
# SIMD-partner priority balancing in the fused kernel: probe + A/B (static 8 GiB, dynamic 64 GiB)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=gpurun_out/r02ai; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step fused_tests 300 python -u -m pytest tests/test_gpu_parity.py -k "test_fused_pass" -x -v --timeout 120 --timeout-method thread || exit 1
step probe_c2 300 python scripts/microbench/fused_probe.py 8 random 4194304 || exit 1
step probe_64 300 python scripts/microbench/fused_probe.py 64 vmimage 4194304 || exit 1
C="PBS_FUSED=0,PBS_BALANCE=0;PBS_FUSED=0,PBS_BALANCE=1;PBS_FUSED=1,PBS_BALANCE=0;PBS_FUSED=1,PBS_BALANCE=1"
step diag_c2 300 env DIAG_CONFIGS="$C" python scripts/pass_diag.py 8 random 4194304 40 || exit 1
step diag_c2_dyn 300 env PBS_SCAN_DYN=1 DIAG_CONFIGS="$C" python scripts/pass_diag.py 8 random 4194304 40 || exit 1
step diag_4m 300 env DIAG_CONFIGS="$C" python scripts/pass_diag.py 64 vmimage 4194304 8 || exit 1
step diag_4m_static 300 env PBS_SCAN_DYN=0 DIAG_CONFIGS="PBS_FUSED=1,PBS_BALANCE=0;PBS_FUSED=1,PBS_BALANCE=1" python scripts/pass_diag.py 64 vmimage 4194304 8 || exit 1
echo done
