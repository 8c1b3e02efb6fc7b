#!/bin/bash
# Round 4a: bench.py verification against the golden cut lists (default line), the
# 7 averages x {VM image, random} table with board power, a zstd phase probe on text/pxar
# with the host libzstd rate, and the scan-pass counter tests.  Each GPU step has its own
# time limit; the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R="$(pwd)"; export TMPDIR=/tmp; O=${OUT:-gpurun_out/r04a}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step tests 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "scan_pass or fused_pass_pool or find_cuts_golden" || exit 1
step bench64 600 python bench.py --cpu-config1 0 || exit 1
step table 900 python scripts/avg_table.py || exit 1
step zstd_probe 400 env PBS_ZSTD_PROBE=1 python3 scripts/zstd_bench.py --corpus text,pxar --gib 1 --reps 2 || exit 1
echo done
