#!/bin/bash
# zstd split kernels + per-workgroup acknowledgements of the scan server: parity first, then
# rates (split vs fused alternating; 64 KiB scan() reads)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r06b}; mkdir -p $O
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step tests_server 300 $PYT -m gpu tests/test_gpu_parity.py -k "server or scan_call or stream" tests/test_examples.py tests/test_shim_sequence.py || exit 1
step tests_zstd 500 $PYT -m gpu tests/test_gpu_zstd.py tests/test_blob_fixture.py tests/test_gpu_blob.py "tests/test_gpu_digest.py::test_upload_stream_host" tests/test_gpu_concurrency.py || exit 1
for i in 1 2; do
  step rate_split_$i 200 env PBS_ZSTD_SPLIT=1 python3 scripts/zstd_bench.py --corpus text,pxar,vm --gib 1 --reps 3 || exit 1
  step rate_fused_$i 200 env PBS_ZSTD_SPLIT=0 python3 scripts/zstd_bench.py --corpus text,pxar,vm --gib 1 --reps 3 || exit 1
done
step probe_split 200 env PBS_ZSTD_PROBE=1 python3 scripts/zstd_bench.py --corpus text,pxar --gib 1 --reps 1 || exit 1
for p in 8192 65536 262144 1048576; do
  step ex_$p 120 examples/test_chunk_speed2 - 1073741824 $p 4194304 0 1 || exit 1
done
step ex_probe_65536 120 env PBS_SERVER_PROBE=1 examples/test_chunk_speed2 - 1073741824 65536 4194304 0 1 || exit 1
step ex_mp1_65536 120 env PBS_SERVER_MINPASS=1 examples/test_chunk_speed2 - 1073741824 65536 4194304 0 1 || exit 1
step ex_mp1_262144 120 env PBS_SERVER_MINPASS=1 examples/test_chunk_speed2 - 1073741824 262144 4194304 0 1 || exit 1
echo done
