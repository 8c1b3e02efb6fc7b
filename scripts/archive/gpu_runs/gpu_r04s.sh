#!/bin/bash
# Round 4s: zstd parse with SIMD-partner balancing (PBS_ZSTD_BALANCE=0: without) -- tests,
# speed A/B alternated, probe.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r04s}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step ztests 400 python -u -m pytest tests/test_gpu_zstd.py -x -v --timeout 200 --timeout-method thread || exit 1
step zbal1 300 python3 scripts/zstd_bench.py --corpus text,pxar --gib 1 --reps 3 || exit 1
step zbal0 300 env PBS_ZSTD_BALANCE=0 python3 scripts/zstd_bench.py --corpus text,pxar --gib 1 --reps 3 || exit 1
step zbal1b 300 python3 scripts/zstd_bench.py --corpus text,pxar --gib 1 --reps 3 || exit 1
step zprobe 300 env PBS_ZSTD_PROBE=1 python3 scripts/zstd_bench.py --corpus text,pxar --gib 1 --reps 1 || exit 1
echo done
