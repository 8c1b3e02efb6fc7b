#!/bin/bash
# fused_publish with 8 exact windows in flight: fused parity, config 2 / 64 KiB / headline split
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=gpurun_out/r02af; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step fused_tests 300 python -u -m pytest tests/test_gpu_parity.py -k fused -x -v --timeout 120 --timeout-method thread || exit 1
step diag_c2 300 python scripts/pass_diag.py 8 random 4194304 50 || exit 1
step diag_64k 300 env PBS_FUSED_MIN_AVG=65536 python scripts/pass_diag.py 64 vmimage 65536 5 || exit 1
step diag_4m 300 python scripts/pass_diag.py 64 vmimage 4194304 10 || exit 1
echo done
