#!/bin/bash
# pipeline: a digest-grid launch skipped while the grid was exiting is retried (next piece,
# upload worker's wait, final drain); digest/pipeline/upload tests, also with a 1 ms idle exit
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r06x}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
step tests 600 $PYT -m gpu tests/test_gpu_digest.py tests/test_gpu_concurrency.py || exit 1
step tests_idle1 600 env PBS_PIPE_IDLE_MS=1 $PYT -m gpu tests/test_gpu_digest.py -k "pipeline or upload" || exit 1
step bench 400 python bench.py || exit 1
echo done
