#!/bin/bash
# Round 4z4: the hybrid digest defaults after the stream A/B (two copy streams, the model's
# D2H cap 50 GB/s): digest tests and the bench's digest stage twice.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r04z4}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
B="python bench.py --steps 3 --warmup 1 --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0 --digest 1"
step tests 400 python -u -m pytest tests/test_gpu_digest.py -x -v --timeout 200 --timeout-method thread || exit 1
step digest_a 300 $B || exit 1
step digest_b 300 $B || exit 1
echo done
