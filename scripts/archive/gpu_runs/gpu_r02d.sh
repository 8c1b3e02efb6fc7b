#!/bin/bash
# fused v2 + scan server: parity subset, unchanged-caller ChunkStream timing, bench lines
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=gpurun_out/r02d; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step fused 300 python -u -m pytest tests/test_gpu_parity.py -k "fused or golden or split or device or small or scan or chunker1 or chunk_stream or speed_loop or invalid" -x -v --timeout 60 --timeout-method thread || exit 1
step ex_8k_unchanged 120 examples/test_chunk_speed2 - 1073741824 8192 4194304 0 1 || exit 1
step ex_256k_unchanged 120 examples/test_chunk_speed2 - 1073741824 262144 4194304 0 1 || exit 1
step ex_8k_gather 120 examples/test_chunk_speed2 - 1073741824 8192 4194304 4194304 1 || exit 1
step ex_8k_unchanged_noserver 120 env PBS_SCAN_SERVER=0 examples/test_chunk_speed2 - 268435456 8192 4194304 0 1 || exit 1
step bench64 300 env PBS_DEBUG_PHASES=1 python bench.py --cpu-baseline 0 --host-inclusive-gib 0 || exit 1
step bench64b 300 python bench.py --cpu-baseline 0 --host-inclusive-gib 0 || exit 1
step c5 300 env PBS_DEBUG_PHASES=1 python bench.py --cpu-baseline 0 --host-inclusive-gib 0 --avg 262144 --steps 3 || exit 1
step bench64_1M 300 env PBS_DEBUG_PHASES=1 python bench.py --cpu-baseline 0 --host-inclusive-gib 0 --avg 1048576 --steps 3 || exit 1

step rocprof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02d/prof -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --cpu-baseline 0 --host-inclusive-gib 0 || exit 1
echo done
