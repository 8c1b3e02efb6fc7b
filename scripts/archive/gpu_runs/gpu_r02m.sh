#!/bin/bash
# zstd blob stage at 64 GiB: bench line + kernel stats
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=gpurun_out/r02m; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step blobs 500 python bench.py --steps 1 --warmup 1 --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0 --blobs 1 || exit 1
step blobs_prof 500 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python bench.py --steps 1 --warmup 1 --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0 --blobs 1 || exit 1
echo done
