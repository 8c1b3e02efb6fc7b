#!/bin/bash
# entropy kernel at four workgroups per CU (23 KiB stream buffer, 128 VGPRs) vs three
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r06aa}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
E4=scripts/ab_libs/e4/libpbschunk.so
step tests_e4 500 env PBS_LIBPBSCHUNK_AB=$E4 $PYT -m gpu tests/test_gpu_zstd.py || exit 1
for r in 1 2; do
  step rate_base_$r 200 python scripts/zstd_bench.py --corpus text,pxar,vm --gib 1 --reps 2 || exit 1
  step rate_e4_$r 200 env PBS_LIBPBSCHUNK_AB=$E4 python scripts/zstd_bench.py --corpus text,pxar,vm --gib 1 --reps 2 || exit 1
done
echo done
