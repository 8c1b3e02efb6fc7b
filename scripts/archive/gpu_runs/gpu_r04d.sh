#!/bin/bash
# Round 4d: lane-measured zstd parse walk (parity vs the twin, then speed + phase probe),
# the 512 KiB fused-pass threshold (scan pass at 256 KiB).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r04d}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step zstd_tests 300 python -u -m pytest tests/test_gpu_zstd.py tests/test_gpu_blob.py -x -v --timeout 200 --timeout-method thread || exit 1
step zstd_probe 400 env PBS_ZSTD_PROBE=1 python3 scripts/zstd_bench.py --corpus text,pxar --gib 1 --reps 2 || exit 1
step zstd_speed 400 python3 scripts/zstd_bench.py --corpus text,pxar,vm --gib 1 --reps 3 || exit 1
step scanpass 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "scan_pass or config5" || exit 1
echo done
