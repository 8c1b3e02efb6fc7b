#!/bin/bash
# Round 3d: scan server v2 (exact_hits per block, staggered multi-wave polling, probe):
# scan()-surface parity tests, then the unchanged caller (one scan() per 8 KiB read,
# test_chunk_speed2 with min_scan 0) with the latency split, for both poll modes.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R="$(pwd)"; export TMPDIR=/tmp; O=${OUT:-gpurun_out/r03d}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step pytest_scan 400 python -u -m pytest tests/test_gpu_parity.py tests/test_examples.py tests/test_gpu_concurrency.py -m gpu -x -v --timeout 300 --timeout-method thread -k "scan or chunk_stream or chunker1 or speed or example or server" || exit 1
step ex_8k_probe 120 env PBS_SERVER_PROBE=1 examples/test_chunk_speed2 - 1073741824 8192 4194304 0 1 || exit 1
step ex_8k_poll1_probe 120 env PBS_SERVER_PROBE=1 PBS_SERVER_POLL=1 examples/test_chunk_speed2 - 1073741824 8192 4194304 0 1 || exit 1
step ex_8k 120 examples/test_chunk_speed2 - 1073741824 8192 4194304 0 1 || exit 1
step ex_256k 120 examples/test_chunk_speed2 - 1073741824 262144 4194304 0 1 || exit 1
echo done
