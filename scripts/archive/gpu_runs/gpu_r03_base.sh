#!/bin/bash
# Round 3 re-entry baseline of the committed code: GPU tests, smoke, headline bench with the
# CPU baseline, rocprofv3 of the same command, zstd corpus + 64 GiB blob stage, the unchanged
# caller's 8 KiB scan() path, configs 2 / 5 and 64 KiB.  Each GPU step has its own limit; the
# script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R="$(pwd)"; export TMPDIR=/tmp; O=${OUT:-gpurun_out/r03_base}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread || exit 1
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step bench64 900 python bench.py || exit 1
step rocprof 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof" -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0 || exit 1
step zstd_corpus 400 python3 scripts/zstd_bench.py --corpus text,pxar,vm --gib 1 --reps 2 || exit 1
step blobs64 600 python bench.py --steps 2 --warmup 1 --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0 --blobs 1 || exit 1
step ex_8k 120 examples/test_chunk_speed2 - 1073741824 8192 4194304 0 1 || exit 1
step ex_8k_probe 120 env PBS_SERVER_PROBE=1 examples/test_chunk_speed2 - 1073741824 8192 4194304 0 1 || exit 1
step c2 300 python bench.py --steps 50 --warmup 30 --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0 --size-gib 8 --workload random || exit 1
step c5 300 python bench.py --steps 10 --warmup 3 --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0 --avg 262144 || exit 1
step a64k 300 python bench.py --steps 5 --warmup 2 --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0 --avg 65536 || exit 1
echo done
