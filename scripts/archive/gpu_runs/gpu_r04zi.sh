#!/bin/bash
# Round 4zi: the sequence bit stream assembled in LDS (ds_or) and stored as whole words
# (no global atomics): zstd GPU tests (byte-equal to the twin), a probe run, and a same-box A/B
# against the committed tree (ab/old), text and pxar.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r04zi}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step tests 400 python -u -m pytest tests/test_gpu_zstd.py -x -v --timeout 200 --timeout-method thread || exit 1
PBS_ZSTD_PROBE=1 step probe 300 python3 scripts/zstd_bench.py --corpus text,pxar --gib 1 --reps 1 || exit 1
for k in 1 2; do
  step old_$k 300 python3 ab/old/scripts/zstd_bench.py --corpus text,pxar --gib 1 --reps 2 || exit 1
  step new_$k 300 python3 scripts/zstd_bench.py --corpus text,pxar --gib 1 --reps 2 || exit 1
done
echo done
