#!/bin/bash
# Round 6, first GPU pass: the new tests (blob fixture, shim replay, bounded waits), the
# whole GPU suite, then the default bench line with the f-stages.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r06a}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
step new_tests 400 $PYT -m gpu tests/test_blob_fixture.py tests/test_shim_sequence.py || exit 1
step gpu_suite 600 $PYT -m gpu tests || exit 1
step bench 600 python bench.py || exit 1
echo done
