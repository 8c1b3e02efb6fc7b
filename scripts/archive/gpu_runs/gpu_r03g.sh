#!/bin/bash
# Round 3g: zstd with workgroup-scope fences; scan server poll A/B.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R="$(pwd)"; export TMPDIR=/tmp; O=${OUT:-gpurun_out/r03g}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step pytest_zstd 400 python -u -m pytest tests/test_gpu_zstd.py -m gpu -x -v --timeout 300 --timeout-method thread || exit 1
step zstd_corpus 400 python -u scripts/zstd_bench.py --gib 1 || exit 1
step blobs64 600 python bench.py --steps 2 --warmup 1 --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0 --blobs 1 || exit 1
step ex_8k_poll4_probe 120 env PBS_SERVER_PROBE=1 PBS_SERVER_POLL=4 examples/test_chunk_speed2 - 1073741824 8192 4194304 0 1 || exit 1
step ex_8k_probe 120 env PBS_SERVER_PROBE=1 examples/test_chunk_speed2 - 1073741824 8192 4194304 0 1 || exit 1
echo done
