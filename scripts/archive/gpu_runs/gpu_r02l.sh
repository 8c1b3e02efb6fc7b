#!/bin/bash
# zstd-1 blob stage: GPU parity against the twin + libzstd decode
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=gpurun_out/r02l; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step zstd_tests 400 python -u -m pytest tests/test_gpu_zstd.py -x -v --timeout 200 --timeout-method thread || exit 1
echo done
