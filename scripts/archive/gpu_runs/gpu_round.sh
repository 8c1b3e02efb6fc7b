#!/bin/bash
# GPU round: tests (incl. slow) -> 64 GiB bench with CPU baseline -> rocprofv3 kernel trace.
# Every GPU step has its own time limit; stops at the first crash/timeout.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R="$(pwd)"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"
  return $rc
}
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  step pytest_gpu 1200 python -m pytest tests -m gpu -x -q; rc=$?
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
step bench64 600 python bench.py --steps ${STEPS:-10} --warmup 2 ${BENCH_ARGS:-} || exit $?
if [ "${PROF:-1}" = "1" ]; then
  step rocprof 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --cpu-baseline 0 --host-inclusive-gib 0 ${BENCH_ARGS:-} || exit $?
fi
exit 0
