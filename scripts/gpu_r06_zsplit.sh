#!/bin/bash
# zstd split kernels: parity (twin byte-equal, decode, the blob fixture, upload path), then
# the corpus rates split vs fused (same box, alternating), and the split probe
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r06_zsplit}; mkdir -p $O
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step tests 500 $PYT -m gpu tests/test_gpu_zstd.py tests/test_blob_fixture.py tests/test_gpu_blob.py "tests/test_gpu_digest.py::test_upload_stream_host" tests/test_gpu_concurrency.py || exit 1
for i in 1 2; do
  step rate_split_$i 200 env PBS_ZSTD_SPLIT=1 python3 scripts/zstd_bench.py --corpus text,pxar,vm --gib 1 --reps 3 || exit 1
  step rate_fused_$i 200 env PBS_ZSTD_SPLIT=0 python3 scripts/zstd_bench.py --corpus text,pxar,vm --gib 1 --reps 3 || exit 1
done
step probe_split 200 env PBS_ZSTD_PROBE=1 python3 scripts/zstd_bench.py --corpus text,pxar --gib 1 --reps 1 || exit 1
echo done
