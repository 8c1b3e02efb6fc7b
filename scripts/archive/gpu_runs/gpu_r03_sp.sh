#!/bin/bash
# Round 3: scan pass for 64 KiB averages (fused scanner, no resolver) + speculative scan server
# probe; the full GPU suite, the 64 KiB / headline / config-5 benches.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r03_sp}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || exit 1
step zstd_corpus 400 env PBS_ZSTD_PROBE=1 python3 scripts/zstd_bench.py --corpus text,pxar,vm --gib 1 --reps 2 || exit 1
step blobs64 600 python bench.py --steps 2 --warmup 1 --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0 --blobs 1 || exit 1
step ex_8k_probe 120 env PBS_SERVER_PROBE=1 examples/test_chunk_speed2 - 1073741824 8192 4194304 0 1 || exit 1
step ex_8k_nospec 120 env PBS_SERVER_SPEC=0 examples/test_chunk_speed2 - 1073741824 8192 4194304 0 1 || exit 1
step a64k 300 python bench.py --steps 5 --warmup 2 --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0 --avg 65536 || exit 1
step a64k_old 300 env PBS_SCAN_PASS=0 python bench.py --steps 5 --warmup 2 --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0 --avg 65536 || exit 1
step bench64 300 python bench.py --steps 10 --warmup 3 --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0 || exit 1
step a128k 300 python bench.py --steps 5 --warmup 2 --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0 --avg 131072 || exit 1
echo done
