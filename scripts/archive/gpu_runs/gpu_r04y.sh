#!/bin/bash
# Round 4y: the new routing defaults (15 MB/s, 10 ms) with the four-lane host SHA-256:
# digest tests, a default-settings sweep, the bench's pipeline stage.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r04y}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step tests 400 python -u -m pytest tests/test_gpu_digest.py tests/test_gpu_concurrency.py -x -v --timeout 200 --timeout-method thread || exit 1
step sweep 600 python scripts/pipe_sweep.py "" "" "" "PBS_SHA_HOST_LANES=1" || exit 1
step bench 600 python bench.py --pipeline-gib 64 || exit 1
echo done
