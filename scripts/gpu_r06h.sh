#!/bin/bash
# zstd split kernels: items dealt by a counter (PBS_ZSTD_DEAL=1, default) vs statically vs the
# fused kernel; corpora text / pxar / VM image and the bench's 64 GiB VM-image blob stage
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r06h}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
step tests_zstd 500 $PYT -m gpu tests/test_gpu_zstd.py tests/test_blob_fixture.py || exit 1
for r in 1 2; do
  step rate_deal_$r 200 env PBS_ZSTD_DEAL=1 python scripts/zstd_bench.py --corpus text,pxar,vm --gib 1 --reps 2 || exit 1
  step rate_static_$r 200 env PBS_ZSTD_DEAL=0 python scripts/zstd_bench.py --corpus text,pxar,vm --gib 1 --reps 2 || exit 1
  step rate_fused_$r 200 env PBS_ZSTD_SPLIT=0 python scripts/zstd_bench.py --corpus text,pxar,vm --gib 1 --reps 2 || exit 1
done
for r in 1 2; do
  step blobs_deal_$r 300 env PBS_ZSTD_DEAL=1 python bench.py --stages 0 --blobs 1 --steps 5 --warmup 2 || exit 1
  step blobs_static_$r 300 env PBS_ZSTD_DEAL=0 python bench.py --stages 0 --blobs 1 --steps 5 --warmup 2 || exit 1
  step blobs_fused_$r 300 env PBS_ZSTD_SPLIT=0 python bench.py --stages 0 --blobs 1 --steps 5 --warmup 2 || exit 1
done
echo done
