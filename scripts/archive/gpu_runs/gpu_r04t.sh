#!/bin/bash
# Round 4t: zstd parse -- does the slower half (waves 4-7) follow the wave or the sub-block?
# PBS_ZSTD_SWAP=1: wave w parses sub-block w ^ 4 (same bytes out: checked by the tests).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r04t}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step ztests_swap 400 env PBS_ZSTD_SWAP=1 python -u -m pytest tests/test_gpu_zstd.py -x -v --timeout 200 --timeout-method thread || exit 1
step zprobe 300 env PBS_ZSTD_PROBE=1 python3 scripts/zstd_bench.py --corpus text,pxar --gib 1 --reps 1 || exit 1
step zprobe_swap 300 env PBS_ZSTD_PROBE=1 PBS_ZSTD_SWAP=1 python3 scripts/zstd_bench.py --corpus text,pxar --gib 1 --reps 1 || exit 1
echo done
