#!/bin/bash
# rocprofv3 kernel-trace stats and a separate FETCH_SIZE PMC pass over bench.py (64 GiB).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R="$(pwd)"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --cpu-baseline 0 --host-inclusive-gib 0 ${BENCH_ARGS:-} > gpurun_out/prof_trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/pmc_fetch" -o run -- python bench.py --steps 3 --warmup 1 --cpu-baseline 0 --host-inclusive-gib 0 ${BENCH_ARGS:-} > gpurun_out/prof_pmc.log 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
python profiles/collect_traffic.py gpurun_out/pmc_fetch > gpurun_out/traffic.log 2>&1
echo "collect rc=$?"
