#!/bin/bash
# Round 4q: scan pass with its resolve right behind the gather (device-side candidate count),
# every gather record at once: parity tests, the split (direct vs copying cut array); zstd with the
# literal mode beside the sequence side: tests, speed, probe.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r04q}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step tests 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_digest.py -x -v --timeout 200 --timeout-method thread -k "scan_pass or pinned or resolve_paths or small_batches or fused or pipeline or full_size" || exit 1
step ztests 400 python -u -m pytest tests/test_gpu_zstd.py tests/test_gpu_concurrency.py -x -v --timeout 200 --timeout-method thread || exit 1
step zspeed 400 python3 scripts/zstd_bench.py --corpus text,pxar,vm --gib 1 --reps 3 || exit 1
step zprobe 400 env PBS_ZSTD_PROBE=1 python3 scripts/zstd_bench.py --corpus text,pxar --gib 1 --reps 2 || exit 1
step split 300 python scripts/scan_pass_split.py || exit 1
step split_copy 300 env PBS_DIRECT_OUT=0 python scripts/scan_pass_split.py --avgs 65536,131072 || exit 1
step conc 300 python scripts/concurrent_pass_ab.py --passes 30 || exit 1
echo done
