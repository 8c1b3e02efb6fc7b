#!/bin/bash
# parse kernel: raw literals of few-sequence blocks copied run by run from the staged window,
# blocks that must go raw written by the parse kernel, the entropy kernel over the listed
# items only, the staged window and hash tables typed as LDS in the parse; tests, corpora, 64 GiB VM blob stage
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r06m}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
step tests_zstd 500 $PYT -m gpu tests/test_gpu_zstd.py tests/test_blob_fixture.py || exit 1
step rate_1 200 python scripts/zstd_bench.py --corpus text,pxar,vm --gib 1 --reps 2 || exit 1
step probe 200 env PBS_ZSTD_PROBE=1 python scripts/zstd_bench.py --corpus vm --gib 1 --reps 1 || exit 1
step blobs_1 300 python bench.py --stages 0 --blobs 1 --steps 5 --warmup 2 || exit 1
step rate_fused 200 env PBS_ZSTD_SPLIT=0 python scripts/zstd_bench.py --corpus text,pxar,vm --gib 1 --reps 2 || exit 1
step rate_2 200 python scripts/zstd_bench.py --corpus text,pxar,vm --gib 1 --reps 2 || exit 1
step blobs_2 300 python bench.py --stages 0 --blobs 1 --steps 5 --warmup 2 || exit 1
echo done
