#!/bin/bash
# fused pass static+balance by default: full GPU suite, size sweep fused vs multi-launch, 64 KiB static vs dynamic
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=gpurun_out/r02ak; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || exit 1
for g in 0.125 0.25 0.5 1 2 4; do step sw_$g 200 env DIAG_CONFIGS="PBS_FUSED=0;PBS_FUSED=1" python scripts/pass_diag.py $g random 4194304 30 || exit 1; done
step a64k 300 env DIAG_CONFIGS="PBS_SCAN_DYN=1;PBS_SCAN_DYN=0" python scripts/pass_diag.py 64 vmimage 65536 5 || exit 1
step c5 300 env DIAG_CONFIGS="PBS_SCAN_DYN=1;PBS_SCAN_DYN=0" python scripts/pass_diag.py 64 vmimage 262144 8 || exit 1
echo done
