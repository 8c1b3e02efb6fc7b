#!/bin/bash
# pipeline host-share threshold sweep with the faster GPU SHA-256
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=gpurun_out/r02k; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
for m in 8 10 12 14; do
  step pipe_min${m} 300 env PBS_PIPE_HOST_MIN=$((m << 20)) python bench.py --steps 1 --warmup 1 --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0 --pipeline-gib 64 || exit 1
done
step pipe_gpu_only 300 env PBS_PIPE_HOST_MIN=0 python bench.py --steps 1 --warmup 1 --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0 --pipeline-gib 64 || exit 1
echo done
