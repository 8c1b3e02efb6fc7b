#!/bin/bash
# Round-5 end artifacts, part B: the digest / blob / pipeline stages, the upload path with
# compression (64 GiB VM image, 16 GiB text- and pxar-like), the examples (the unchanged caller
# at 8 KiB, 64 KiB, 256 KiB and 1 MiB reads beside the gathering one) and the zstd corpora.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R="$(pwd)"; export TMPDIR=/tmp; O=${OUT:-gpurun_out/final_r05}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
NOEXTRA="--cpu-baseline 0 --cpu-config1 0 --host-inclusive-gib 0 --secondary-random 0"
step stages 300 python bench.py --steps 3 --warmup 1 $NOEXTRA --digest 1 --blobs 1 --pipeline-gib 64 || exit 1
step upload_vm 300 python bench.py --steps 2 --warmup 1 $NOEXTRA --upload-gib 64 || exit 1
step upload_text 300 python bench.py --steps 2 --warmup 1 $NOEXTRA --upload-gib 16 --upload-corpus text || exit 1
step upload_pxar 300 python bench.py --steps 2 --warmup 1 $NOEXTRA --upload-gib 16 --upload-corpus pxar || exit 1
step examples 200 bash -c "examples/test_chunk_speed && examples/test_chunk_speed2 - 1073741824 8192 4194304 0 1 && examples/test_chunk_size | tail -3" || exit 1
for p in 65536 262144 1048576; do step ex_$p 120 examples/test_chunk_speed2 - 1073741824 $p 4194304 0 1 || exit 1; done
step zstd_corpus 300 python3 scripts/zstd_bench.py --corpus text,pxar,vm --gib 1 --reps 2 || exit 1
echo done
