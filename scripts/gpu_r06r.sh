#!/bin/bash
# history rounds sampling at least every 2nd position after a hit (PBS_ZHIST_MIN=2 build) vs 1
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r06r}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
for r in 1 2; do
  step rate_base_$r 200 python scripts/zstd_bench.py --corpus text,pxar,vm --gib 1 --reps 2 || exit 1
  step rate_hmin2_$r 200 env PBS_LIBPBSCHUNK_AB=scripts/ab_libs/hmin2/libpbschunk.so python scripts/zstd_bench.py --corpus text,pxar,vm --gib 1 --reps 2 || exit 1
done
step probe_hmin2 200 env PBS_ZSTD_PROBE=1 PBS_LIBPBSCHUNK_AB=scripts/ab_libs/hmin2/libpbschunk.so python scripts/zstd_bench.py --corpus text --gib 1 --reps 1 || exit 1
echo done
