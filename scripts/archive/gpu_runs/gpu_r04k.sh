#!/bin/bash
# Round 4k: pipeline work area kept between calls: digest tests, repeated sweep calls, bench pipeline stage.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r04k}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step tests 400 python -u -m pytest tests/test_gpu_digest.py tests/test_gpu_concurrency.py tests/test_examples.py -x -v --timeout 200 --timeout-method thread || exit 1
step ex 120 examples/test_chunk_speed2 - 1073741824 8192 4194304 0 1 || exit 1
step sweep 600 python scripts/pipe_sweep.py "" "" "" || exit 1
step split 300 python scripts/scan_pass_split.py || exit 1
step fusedlag 300 env PBS_DEBUG_PHASES=1 PBS_FUSED=1 python scripts/scan_pass_split.py --avgs 131072,262144,1048576,4194304 --steps 3 || exit 1
step bench 600 python bench.py --pipeline-gib 64 || exit 1
echo done
