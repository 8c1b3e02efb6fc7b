#!/bin/bash
# Round 3: zstd literal runs copied dword by dword in one pass, raw blocks by dwords, history
# rounds from step 4: parity with the twin, corpus ratio/throughput, 64 GiB blob stage (+probe).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r03_z}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step pytest_zstd 400 python -u -m pytest tests/test_gpu_zstd.py tests/test_gpu_blob.py -m gpu -x -v --timeout 300 --timeout-method thread || exit 1
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step zstd_corpus 400 python3 scripts/zstd_bench.py --corpus text,pxar,vm --gib 1 --reps 2 || exit 1
step blobs64 600 python bench.py --steps 2 --warmup 1 --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0 --blobs 1 || exit 1
step blobs64_probe 600 env PBS_ZSTD_PROBE=1 python bench.py --steps 1 --warmup 1 --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0 --blobs 1 || exit 1
echo done
