#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r06f}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
step tests_dbl0 400 env PBS_ZSTD_DBL=0 $PYT -m gpu tests/test_gpu_zstd.py tests/test_blob_fixture.py || exit 1
step tests_default 400 $PYT -m gpu tests/test_gpu_zstd.py || exit 1
for i in 1 2; do
for d in 0 24 100000; do
step rate_dbl${d}_$i 200 env PBS_ZSTD_DBL=$d python3 scripts/zstd_bench.py --corpus text,pxar,vm --gib 1 --reps 3 || exit 1
done
done
step probe 200 env PBS_ZSTD_PROBE=1 python3 scripts/zstd_bench.py --corpus text,pxar --gib 1 --reps 1 || exit 1
echo done
