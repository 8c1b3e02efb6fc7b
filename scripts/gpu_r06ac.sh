#!/bin/bash
# parse kernel: the repeat coding from records held in registers, the code histogram from the final codes

cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r06ac}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
step tests_zstd 500 $PYT -m gpu tests/test_gpu_zstd.py tests/test_blob_fixture.py || exit 1
step rate_1 200 python scripts/zstd_bench.py --corpus text,pxar,vm --gib 1 --reps 2 || exit 1
step probe 200 env PBS_ZSTD_PROBE=1 python scripts/zstd_bench.py --corpus text --gib 1 --reps 1 || exit 1
step rate_2 200 python scripts/zstd_bench.py --corpus text,pxar,vm --gib 1 --reps 2 || exit 1
echo done
