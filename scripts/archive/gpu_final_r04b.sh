#!/bin/bash
# Round-4 end artifacts, part B: the digest / blob / pipeline stages, examples (the
# unchanged caller beside the gathering one), the zstd corpora, configs 2 and 5, 64 KiB,
# and the table of every legal average x {VM image, random} with board power.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R="$(pwd)"; export TMPDIR=/tmp; O=${OUT:-gpurun_out/final_r04}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step stages 300 python bench.py --steps 3 --warmup 1 --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0 --digest 1 --blobs 1 --pipeline-gib 64 || exit 1
step examples 200 bash -c "examples/test_chunk_speed && examples/test_chunk_speed2 - 1073741824 8192 4194304 0 1 && examples/test_chunk_size | tail -3" || exit 1
step ex_256k 120 examples/test_chunk_speed2 - 1073741824 262144 4194304 0 1 || exit 1
step zstd_corpus 300 python3 scripts/zstd_bench.py --corpus text,pxar,vm --gib 1 --reps 2 || exit 1
step c2 200 python bench.py --steps 50 --warmup 30 --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0 --size-gib 8 --workload random || exit 1
step c5 200 python bench.py --steps 10 --warmup 3 --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0 --avg 262144 || exit 1
step table 500 python scripts/avg_table.py || exit 1
step c2power 200 python scripts/avg_table.py --kinds random --avgs 4194304 --size-gib 8 --steps 50 --warmup 30 || exit 1
echo done
