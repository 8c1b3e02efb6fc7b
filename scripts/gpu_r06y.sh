#!/bin/bash
# zstd: many batches per call and both dealings against the twin
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r06y}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
step tests_zstd 500 $PYT -m gpu tests/test_gpu_zstd.py || exit 1
echo done
