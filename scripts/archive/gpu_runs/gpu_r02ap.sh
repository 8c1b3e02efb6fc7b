#!/bin/bash
# static rounds + dynamic pool of short tiles: parity, probe, pool sweeps
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=gpurun_out/r02ap; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step fused_tests 600 python -u -m pytest tests/test_gpu_parity.py -k "fused or golden or split" -x -v --timeout 300 --timeout-method thread || exit 1
step probe_c2 200 python scripts/microbench/fused_probe.py 8 random 4194304 || exit 1
C="PBS_SCAN_DYN=1,PBS_POOL_PCT=0;PBS_SCAN_DYN=0,PBS_POOL_PCT=0;PBS_SCAN_DYN=0,PBS_POOL_PCT=25,PBS_POOL_DIV=8;PBS_SCAN_DYN=0,PBS_POOL_PCT=25,PBS_POOL_DIV=4;PBS_SCAN_DYN=0,PBS_POOL_PCT=12,PBS_POOL_DIV=4;PBS_SCAN_DYN=0,PBS_POOL_PCT=40,PBS_POOL_DIV=4"
step c3 400 env DIAG_CONFIGS="$C" python scripts/pass_diag.py 64 vmimage 4194304 5 || exit 1
step c2 300 env PBS_FUSED=1 DIAG_CONFIGS="$C" python scripts/pass_diag.py 8 random 4194304 30 || exit 1
step c5 400 env PBS_FUSED=1 DIAG_CONFIGS="$C" python scripts/pass_diag.py 64 vmimage 262144 5 || exit 1
echo done
