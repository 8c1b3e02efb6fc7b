#!/bin/bash
# SHA-256 split kernel with three W slots (rounds wave prefetches the next block's W+K)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=gpurun_out/r02h; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step digest_tests 500 python -u -m pytest tests/test_gpu_digest.py -x -v --timeout 300 --timeout-method thread || exit 1
step digest 400 python bench.py --steps 2 --warmup 1 --cpu-baseline 0 --host-inclusive-gib 0 --digest 1 || exit 1
for m in 6 7 9; do
  step pipe_min${m} 300 env PBS_PIPE_HOST_MIN=$((m << 20)) python bench.py --steps 1 --warmup 1 --cpu-baseline 0 --host-inclusive-gib 0 --pipeline-gib 64 || exit 1
done
step pipe_t16 300 env PBS_PIPE_HOST_THREADS=16 python bench.py --steps 1 --warmup 1 --cpu-baseline 0 --host-inclusive-gib 0 --pipeline-gib 64 || exit 1
echo done
