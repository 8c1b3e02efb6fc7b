#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r06e}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
step tests_zstd 500 $PYT -m gpu tests/test_gpu_zstd.py tests/test_blob_fixture.py tests/test_gpu_concurrency.py "tests/test_gpu_digest.py::test_upload_stream_mixed_compressed" || exit 1
for i in 1 2; do
step rate_overlap_$i 200 env PBS_ZSTD_OVERLAP=1 python3 scripts/zstd_bench.py --corpus text,pxar,vm --gib 1 --reps 3 || exit 1
step rate_serial_$i 200 env PBS_ZSTD_OVERLAP=0 python3 scripts/zstd_bench.py --corpus text,pxar,vm --gib 1 --reps 3 || exit 1
done
step rate_serial8k 200 env PBS_ZSTD_OVERLAP=0 PBS_ZSTD_BATCH=8192 python3 scripts/zstd_bench.py --corpus text,pxar,vm --gib 1 --reps 3 || exit 1
step trace 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 scripts/zstd_bench.py --corpus text --gib 1 --reps 2 || exit 1
echo done
