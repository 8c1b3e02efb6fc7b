#!/bin/bash
# Round 4zb: same-box A/B of the zstd walk change: the committed tree (ab/old, built there)
# vs the working tree, alternated, text and pxar corpora.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r04zb}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
R=$(pwd)
for k in 1 2; do
  step old_$k 300 python3 ab/old/scripts/zstd_bench.py --corpus text,pxar --gib 1 --reps 2 || exit 1
  step new_$k 300 python3 scripts/zstd_bench.py --corpus text,pxar --gib 1 --reps 2 || exit 1
done
echo done
