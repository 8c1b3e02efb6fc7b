#!/bin/bash
# Round 3a: mailbox latency microbenchmark (scan() per 8 KiB read), then the GPU tests
# that changed this round (multi-rank rehearsal with per-rank oracle diffs in both modes,
# RCCL world-1 bench, concurrent handles, digest / blob / zstd after the device-guard
# fixes) and the rest of the non-slow GPU suite.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R="$(pwd)"; export TMPDIR=/tmp; O=${OUT:-gpurun_out/r03a}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
SKIP_NEW=${SKIP_NEW:-0}; [ "$SKIP_NEW" = 1 ] || step pytest_new 600 python -u -m pytest tests/test_dist.py tests/test_gpu_concurrency.py tests/test_gpu_digest.py tests/test_gpu_blob.py -m gpu -x -v --timeout 300 --timeout-method thread || exit 1
step pytest_rest 900 python -u -m pytest tests -m "gpu and not slow" -x -v --timeout 300 --timeout-method thread --deselect tests/test_gpu_concurrency.py --ignore tests/test_gpu_zstd.py --ignore tests/test_dist.py || exit 1
step mailbox 90 scripts/microbench/mb_mailbox || exit 1
echo done
