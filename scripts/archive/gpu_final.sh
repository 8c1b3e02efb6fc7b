#!/bin/bash
# Round-end artifacts: GPU tests, smoke, PMC traffic, headline bench (with CPU baseline
# and host-inclusive rate), rocprofv3 kernel stats of the same command, digest stage,
# configs 2 and 5.  Each GPU step has its own time limit; the script stops at the first
# failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R="$(pwd)"; export TMPDIR=/tmp; mkdir -p gpurun_out/final
O=gpurun_out/final
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 300 || exit 1
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step pmc 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/$O/pmc_fetch" -o run -- python bench.py --steps 3 --warmup 1 --cpu-baseline 0 --host-inclusive-gib 0 || exit 1
python profiles/collect_traffic.py "$O/pmc_fetch" --out "$O/traffic.json" > "$O/collect.log" 2>&1 && cp "$O/traffic.json" profiles/traffic_latest.json
step bench64 600 python bench.py || exit 1
step rocprof 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof" -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --cpu-baseline 0 --host-inclusive-gib 0 || exit 1
step digest 400 python bench.py --steps 3 --warmup 1 --cpu-baseline 0 --host-inclusive-gib 0 --digest 1 || exit 1
step rocprof_digest 400 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_digest" -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --cpu-baseline 0 --host-inclusive-gib 0 --digest 1 || exit 1
step pmc_crc 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/$O/pmc_crc" -o run -- python bench.py --steps 1 --warmup 0 --cpu-baseline 0 --host-inclusive-gib 0 --digest 1 || exit 1
python profiles/collect_traffic.py "$O/pmc_crc" --kernel crc32_chunks_kernel --out "$O/traffic_crc.json" > "$O/collect_crc.log" 2>&1
step examples 300 bash -c "make -s -C examples && examples/test_chunk_speed && examples/test_chunk_speed2 | tail -3 && examples/test_chunk_size | tail -3" || exit 1
step c2 300 python bench.py --steps 50 --warmup 30 --cpu-baseline 0 --host-inclusive-gib 0 --size-gib 8 --workload random || exit 1
step c5 300 python bench.py --steps 10 --warmup 3 --cpu-baseline 0 --host-inclusive-gib 0 --avg 262144 || exit 1
echo done
