#!/bin/bash
# zstd phase probe of the current build (workgroup 0), text and pxar corpora at 1 GiB
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r06_zprobe}; mkdir -p $O
timeout -k 10 300 env PBS_ZSTD_PROBE=1 python3 scripts/zstd_bench.py --corpus text,pxar --gib 1 --reps 1 > $O/probe.log 2>&1 || exit 1
timeout -k 10 300 python3 scripts/zstd_bench.py --corpus text,pxar --gib 1 --reps 3 > $O/rate.log 2>&1 || exit 1
echo done
