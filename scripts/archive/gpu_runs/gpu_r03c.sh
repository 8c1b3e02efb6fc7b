#!/bin/bash
# Round 3c: mailbox latency (multi-wave polling), the blob stage on the 64 GiB VM image
# (bench --blobs) and on text / pxar corpora (scripts/zstd_bench.py).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R="$(pwd)"; export TMPDIR=/tmp; O=${OUT:-gpurun_out/r03c}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step mailbox 90 scripts/microbench/mb_mailbox || exit 1
step zstd_corpus 400 python -u scripts/zstd_bench.py --gib 1 || exit 1
step blobs64 600 python bench.py --steps 2 --warmup 1 --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0 --blobs 1 || exit 1
echo done
