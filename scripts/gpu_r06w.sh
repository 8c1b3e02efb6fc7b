#!/bin/bash
# the adopted window / history step: zstd + blob + upload tests (twin byte-equal), corpora
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r06w}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
step tests 600 $PYT -m gpu tests/test_gpu_zstd.py tests/test_blob_fixture.py tests/test_gpu_digest.py -k "zstd or blob or upload" || exit 1
step rate 200 python scripts/zstd_bench.py --corpus text,pxar,vm --gib 1 --reps 2 || exit 1
echo done
