#!/bin/bash
# SIMD balancing modes (0 off, 1 priority, 2 priority + yield): probe pair gaps, 64 GiB static vs dynamic, 8 GiB
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=gpurun_out/r02aj; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
for b in 0 1 2; do step probe_c2_b$b 200 env PBS_BALANCE=$b python scripts/microbench/fused_probe.py 8 random 4194304 || exit 1; done
step probe_64s_b1 200 env PBS_BALANCE=1 PBS_SCAN_DYN=0 python scripts/microbench/fused_probe.py 64 vmimage 4194304 || exit 1
C="PBS_SCAN_DYN=1,PBS_BALANCE=0;PBS_SCAN_DYN=0,PBS_BALANCE=1;PBS_SCAN_DYN=0,PBS_BALANCE=2"
step diag_4m 300 env PBS_FUSED=1 DIAG_CONFIGS="$C" python scripts/pass_diag.py 64 vmimage 4194304 8 || exit 1
step diag_r64 300 env PBS_FUSED=1 DIAG_CONFIGS="$C" python scripts/pass_diag.py 64 random 4194304 5 || exit 1
step diag_c2 300 env PBS_FUSED=1 DIAG_CONFIGS="PBS_BALANCE=0;PBS_BALANCE=1;PBS_BALANCE=2" python scripts/pass_diag.py 8 random 4194304 40 || exit 1
echo done
