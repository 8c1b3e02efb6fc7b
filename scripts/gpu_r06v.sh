#!/bin/bash
# parse variants: history sampling step after a hit (1 / 2) x sub-block window (16 / 12 / 8 KiB)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r06v}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
for r in 1 2; do
  step rate_base_$r 200 python scripts/zstd_bench.py --corpus text,pxar,vm --gib 1 --reps 2 || exit 1
  for v in h2w16 h2w12 h1w12 h2w8; do
    step rate_${v}_$r 200 env PBS_LIBPBSCHUNK_AB=scripts/ab_libs/$v/libpbschunk.so python scripts/zstd_bench.py --corpus text,pxar,vm --gib 1 --reps 2 || exit 1
  done
done
echo done
