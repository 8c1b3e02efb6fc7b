#!/bin/bash
# Round-3 end artifacts: GPU tests, smoke, PMC traffic of the fused kernel (before the bench,
# so the bench line carries it), headline bench with CPU baseline / config-1 sample /
# host-inclusive rate / random-data secondary line, rocprofv3 kernel stats of the same
# command, digest + blob + pipeline stages, configs 2 and 5, 64 KiB, examples.  Each GPU
# step has its own time limit; the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R="$(pwd)"; export TMPDIR=/tmp; O=${OUT:-gpurun_out/final_r03}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread || exit 1
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step pmc 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/$O/pmc_fetch" -o run -- python bench.py --steps 3 --warmup 1 --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0 || exit 1
python profiles/collect_traffic.py "$O/pmc_fetch" --out "$O/traffic.json" > "$O/collect.log" 2>&1 && cp "$O/traffic.json" profiles/traffic_latest.json
step bench64 900 python bench.py || exit 1
step rocprof 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof" -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0 || exit 1
step stages 600 python bench.py --steps 3 --warmup 1 --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0 --digest 1 --blobs 1 --pipeline-gib 64 || exit 1
step rocprof_stages 600 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_stages" -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0 --digest 1 --blobs 1 || exit 1
step examples 300 bash -c "examples/test_chunk_speed && examples/test_chunk_speed2 | tail -3 && examples/test_chunk_size | tail -3" || exit 1
step ex_8k 120 examples/test_chunk_speed2 - 1073741824 8192 4194304 0 1 || exit 1
step ex_8k_probe 120 env PBS_SERVER_PROBE=1 examples/test_chunk_speed2 - 1073741824 8192 4194304 0 1 || exit 1
step ex_256k 120 examples/test_chunk_speed2 - 1073741824 262144 4194304 0 1 || exit 1
step zstd_corpus 400 python3 scripts/zstd_bench.py --corpus text,pxar,vm --gib 1 --reps 2 || exit 1
step c2 300 python bench.py --steps 50 --warmup 30 --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0 --size-gib 8 --workload random || exit 1
step c5 300 python bench.py --steps 10 --warmup 3 --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0 --avg 262144 || exit 1
step a64k 300 python bench.py --steps 5 --warmup 2 --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0 --avg 65536 || exit 1
echo done
