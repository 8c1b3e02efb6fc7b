#!/bin/bash
# Round 3: host<->kernel mailbox latency split (mb_poll), zstd phase probe on the VM image.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r03_poll}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step mb_poll 120 scripts/microbench/mb_poll || exit 1
step zstd_probe_vm 300 env PBS_ZSTD_PROBE=1 python3 scripts/zstd_bench.py --corpus vm,text --gib 1 --reps 1 || exit 1
step blobs64_probe 600 env PBS_ZSTD_PROBE=1 python bench.py --steps 1 --warmup 1 --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0 --blobs 1 || exit 1
echo done
