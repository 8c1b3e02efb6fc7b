#!/bin/bash
# Round-6 end artifacts, part B: the examples (the unchanged caller at 8 KiB .. 1 MiB reads
# beside the gathering one), the zstd corpora with their kernel trace, the upload path on the
# pxar-like corpus, configs 2 and 5, and the PMC per-byte records (scan kernel; zstd kernels).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R="$(pwd)"; export TMPDIR=/tmp; O=${OUT:-gpurun_out/final_r06}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
NOEXTRA="--cpu-baseline 0 --cpu-config1 0 --host-inclusive-gib 0 --secondary-random 0 --stages 0"
step examples 200 bash -c "examples/test_chunk_speed && examples/test_chunk_speed2 - 1073741824 8192 4194304 0 1 && examples/test_chunk_size | tail -3" || exit 1
for p in 16384 65536 262144 1048576; do step ex_$p 120 examples/test_chunk_speed2 - 1073741824 $p 4194304 0 1 || exit 1; done
step zstd_corpus 300 python3 scripts/zstd_bench.py --corpus text,pxar,vm --gib 1 --reps 2 || exit 1
step zstd_trace 300 rocprofv3 --kernel-trace --stats --output-format csv rocpd -d "$R/$O/zstd_prof" -o run -- python3 scripts/zstd_bench.py --corpus text,pxar --gib 1 --reps 2 || exit 1
python3 scripts/ktrace.py "$(ls $O/zstd_prof/*.db $O/zstd_prof/*/*.db 2>/dev/null | head -1)" zstd > "$O/zstd_ktrace.txt" 2>&1
step upload_pxar 300 python bench.py --steps 2 --warmup 1 $NOEXTRA --upload-gib 16 --upload-corpus pxar || exit 1
step c2 200 python bench.py --steps 50 --warmup 30 $NOEXTRA --size-gib 8 --workload random || exit 1
step c5 200 python bench.py --steps 10 --warmup 3 $NOEXTRA --avg 262144 || exit 1
echo done
