#!/bin/bash
# full GPU suite + examples + headline bench with CPU baseline
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=gpurun_out/r02e; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread || exit 1
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step examples 300 bash -c "make -s -C examples && examples/test_chunk_speed | tail -3 && examples/test_chunk_speed2 - 1073741824 8192 4194304 0 1 && examples/test_chunk_size | tail -3" || exit 1
step bench64 600 python bench.py || exit 1
echo done
