#!/bin/bash
# Round 4g: the host-stream pipeline with the persistent digest queue and deadline routing:
# parity tests, then the 64 GiB stage (and the fixed 8 MiB threshold for A/B).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r04g}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step tests 300 python -u -m pytest tests/test_gpu_digest.py -x -v --timeout 200 --timeout-method thread -k "pipeline or upload" || exit 1
step pipe 400 python bench.py --steps 2 --warmup 1 --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0 --pipeline-gib 64 || exit 1
step pipe_fixed8 400 env PBS_PIPE_HOST_MIN=8388608 python bench.py --steps 2 --warmup 1 --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0 --pipeline-gib 64 || exit 1
echo done
