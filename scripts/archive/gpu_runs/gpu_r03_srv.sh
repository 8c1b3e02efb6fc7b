#!/bin/bash
# Round 3: scan server v3 (chain rows, no per-lane warm-up): scan() parity, the unchanged
# caller's 8 KiB and 256 KiB reads with the phase probe.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r03_srv}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step pytest_scan 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_concurrency.py tests/test_examples.py -m gpu -x -v --timeout 200 --timeout-method thread -k "scan or chunk_stream or chunker1 or chunk_speed or concurren or example" || exit 1
step ex_8k 120 examples/test_chunk_speed2 - 1073741824 8192 4194304 0 1 || exit 1
step ex_8k_b 120 examples/test_chunk_speed2 - 1073741824 8192 4194304 0 1 || exit 1
step ex_8k_probe 120 env PBS_SERVER_PROBE=1 examples/test_chunk_speed2 - 1073741824 8192 4194304 0 1 || exit 1
step ex_8k_nospec 120 env PBS_SERVER_SPEC=0 examples/test_chunk_speed2 - 1073741824 8192 4194304 0 1 || exit 1
step ex_256k 120 examples/test_chunk_speed2 - 1073741824 262144 4194304 0 1 || exit 1
step ex_256k_probe 120 env PBS_SERVER_PROBE=1 examples/test_chunk_speed2 - 1073741824 262144 4194304 0 1 || exit 1
step ex_256k_nospec 120 env PBS_SERVER_SPEC=0 examples/test_chunk_speed2 - 1073741824 262144 4194304 0 1 || exit 1
step ex_64k 120 examples/test_chunk_speed2 - 1073741824 65536 4194304 0 1 || exit 1
echo done
