#!/bin/bash
# hybrid SHA-256 (host SHA extensions for the longest chunks) and the pipeline's host share
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=gpurun_out/r02g; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
lscpu > $O/lscpu.txt 2>&1; cat /sys/fs/cgroup/cpu.max > $O/cpu_max.txt 2>&1
step digest_tests 500 python -u -m pytest tests/test_gpu_digest.py -x -v --timeout 300 --timeout-method thread || exit 1
step digest 400 python bench.py --steps 2 --warmup 1 --cpu-baseline 0 --host-inclusive-gib 0 --digest 1 || exit 1
step pipeline 400 python bench.py --steps 2 --warmup 1 --cpu-baseline 0 --host-inclusive-gib 0 --pipeline-gib 64 || exit 1
step pipeline_gpu_only 400 env PBS_PIPE_HOST_MIN=0 python bench.py --steps 2 --warmup 1 --cpu-baseline 0 --host-inclusive-gib 0 --pipeline-gib 64 || exit 1
echo done
