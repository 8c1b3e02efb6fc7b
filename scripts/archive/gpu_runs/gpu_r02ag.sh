#!/bin/bash
# fused pass, static order with runtime segment lengths: parity, then multi-launch vs fused by size
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=gpurun_out/r02ag; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step fused_tests 600 python -u -m pytest tests/test_gpu_parity.py -k "fused" -x -v --timeout 300 --timeout-method thread || exit 1
step diag_c2 300 python scripts/pass_diag.py 8 random 4194304 50 || exit 1
step diag_4m 300 python scripts/pass_diag.py 64 vmimage 4194304 10 || exit 1
for g in 1 2 4 16; do step diag_r$g 300 python scripts/pass_diag.py $g random 4194304 30 || exit 1; done
step diag_vm8 300 python scripts/pass_diag.py 8 vmimage 4194304 30 || exit 1
step diag_c5_8 300 python scripts/pass_diag.py 8 vmimage 262144 30 || exit 1
echo done
