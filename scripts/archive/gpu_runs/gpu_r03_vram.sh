#!/bin/bash
# scan server request record + slot in BAR-written VRAM: scan() parity tests, the
# concurrency test, and test_chunk_speed2 over 8 KiB / 256 KiB reads in both placements.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=${OUT:-gpurun_out/vram}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step pytest_scan 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_concurrency.py tests/test_examples.py -m gpu -v --timeout 120 --timeout-method thread -k "scan or chunker1 or chunk_stream or concurrency or server or example or speed" || exit 1
for v in 1 0 1 0; do k=$((k+1));
  step ex_8k_vram${v}_$k 120 env PBS_SERVER_VRAM=$v examples/test_chunk_speed2 - 1073741824 8192 4194304 0 1 || exit 1
done
step ex_8k_probe_vram1 120 env PBS_SERVER_PROBE=1 examples/test_chunk_speed2 - 1073741824 8192 4194304 0 1 || exit 1
step ex_8k_probe_vram0 120 env PBS_SERVER_VRAM=0 PBS_SERVER_PROBE=1 examples/test_chunk_speed2 - 1073741824 8192 4194304 0 1 || exit 1
step ex_256k_vram1 120 examples/test_chunk_speed2 - 1073741824 262144 4194304 0 1 || exit 1
step ex_256k_vram0 120 env PBS_SERVER_VRAM=0 examples/test_chunk_speed2 - 1073741824 262144 4194304 0 1 || exit 1
echo done
