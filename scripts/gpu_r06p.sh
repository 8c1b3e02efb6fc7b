#!/bin/bash
# zstd batch size (items per parse/entropy launch pair): 4096 / 8192 (default) / 16384 / 32768
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r06p}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
for r in 1 2; do
  for b in 4096 8192 16384 32768; do
    step rate_b${b}_$r 200 env PBS_ZSTD_BATCH=$b python scripts/zstd_bench.py --corpus text,pxar,vm --gib 1 --reps 2 || exit 1
  done
done
echo done
