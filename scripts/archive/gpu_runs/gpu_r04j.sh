#!/bin/bash
# Round 4j: digest/pipeline/blob/concurrency tests with the digest queue defaults, and the
# 64 GiB pipeline stage twice.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r04j}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step tests 400 python -u -m pytest tests/test_gpu_digest.py tests/test_gpu_blob.py tests/test_gpu_concurrency.py tests/test_gpu_zstd.py -x -v --timeout 200 --timeout-method thread || exit 1
step sweep 600 python scripts/pipe_sweep.py "" "" || exit 1
echo done
