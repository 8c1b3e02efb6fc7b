#!/bin/bash
# diagnostic: one zstd GPU test with the HIP runtime's error log
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r06ad}; mkdir -p $O
timeout -k 10 200 env AMD_LOG_LEVEL=1 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_zstd.py -k "mixed_chunks and 0" > $O/t.log 2>&1; echo rc=$?
