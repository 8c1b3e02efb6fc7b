#!/bin/bash
# zstd blob stage: staging loads in flight + metadata prefetch; phase probe
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=gpurun_out/r02ab; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step zstd_tests 400 python -u -m pytest tests/test_gpu_zstd.py -x -v --timeout 200 --timeout-method thread || exit 1
step blobs 500 python bench.py --steps 1 --warmup 1 --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0 --blobs 1 || exit 1
step probe 500 env PBS_ZSTD_PROBE=1 python bench.py --steps 1 --warmup 1 --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0 --blobs 1 || exit 1
echo done
