#!/bin/bash
# Round 3: relaxed vs release acknowledgement (mb_poll), the server with a relaxed ack when no
# candidates were stored: scan() parity and the unchanged caller's 8 KiB reads.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r03_ack}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step mb_poll 120 scripts/microbench/mb_poll || exit 1
step pytest_scan 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_concurrency.py tests/test_examples.py -m gpu -x -v --timeout 200 --timeout-method thread -k "scan or chunk_stream or chunker1 or chunk_speed or concurren or example" || exit 1
step ex_8k 120 examples/test_chunk_speed2 - 1073741824 8192 4194304 0 1 || exit 1
step ex_8k_b 120 examples/test_chunk_speed2 - 1073741824 8192 4194304 0 1 || exit 1
step ex_8k_probe 120 env PBS_SERVER_PROBE=1 examples/test_chunk_speed2 - 1073741824 8192 4194304 0 1 || exit 1
echo done
