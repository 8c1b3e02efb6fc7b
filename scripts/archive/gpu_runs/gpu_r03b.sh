#!/bin/bash
# Round 3b: the zstd v2 blob encoder (Huffman literals, FSE sequence tables, repeat codes,
# 8 KiB sub-blocks with a 16 KiB window) against its twin, then the rest of the GPU suite
# and the mailbox latency microbenchmark.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R="$(pwd)"; export TMPDIR=/tmp; O=${OUT:-gpurun_out/r03b}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step pytest_zstd 400 python -u -m pytest tests/test_gpu_zstd.py tests/test_gpu_blob.py -m gpu -x -v --timeout 300 --timeout-method thread || exit 1
step pytest_rest 900 python -u -m pytest tests -m "gpu and not slow" -x -v --timeout 300 --timeout-method thread --ignore tests/test_gpu_zstd.py --ignore tests/test_gpu_blob.py --ignore tests/test_dist.py --ignore tests/test_gpu_concurrency.py || exit 1
step mailbox 90 scripts/microbench/mb_mailbox || exit 1
echo done
