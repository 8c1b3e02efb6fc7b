#!/bin/bash
# Round 4r: zstd -- per-stream code histograms privatised (16 copies) and batched.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r04r}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step ztests 400 python -u -m pytest tests/test_gpu_zstd.py -x -v --timeout 200 --timeout-method thread || exit 1
step zspeed 400 python3 scripts/zstd_bench.py --corpus text,pxar,vm --gib 1 --reps 3 || exit 1
step zprobe 400 env PBS_ZSTD_PROBE=1 python3 scripts/zstd_bench.py --corpus text,pxar --gib 1 --reps 1 || exit 1
echo done
