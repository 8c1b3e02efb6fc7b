#!/bin/bash
# Round 4za: zstd walk step tests as one byte per lane with wave-uniform lane ranges (masks
# on the scalar unit): zstd GPU tests (frames byte-equal to the twin), the corpora bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r04za}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step tests 500 python -u -m pytest tests/test_gpu_zstd.py -x -v --timeout 300 --timeout-method thread || exit 1
step corpus 300 python3 scripts/zstd_bench.py --corpus text,pxar --gib 1 --reps 2 || exit 1
echo done
