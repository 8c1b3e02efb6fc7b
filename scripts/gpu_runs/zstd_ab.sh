#!/bin/bash
# zstd A/B on one box: the zstd GPU tests with the in-tree build, then the corpora rates
# alternating the saved baseline (scripts/ab_libs/libpbschunk_base.so) and the tree.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/zstd_ab
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_zstd.py > $OUT/tests.log 2>&1 || exit $?
for i in 1 2; do
  PBS_LIBPBSCHUNK_AB=$(pwd)/scripts/ab_libs/libpbschunk_base.so timeout -k 10 120 python -u scripts/zstd_ab.py >> $OUT/base.log 2>&1 || exit $?
  timeout -k 10 120 python -u scripts/zstd_ab.py >> $OUT/new.log 2>&1 || exit $?
done
PBS_ZSTD_PROBE=1 timeout -k 10 120 python -u scripts/zstd_ab.py --reps 1 > $OUT/probe.log 2>&1
