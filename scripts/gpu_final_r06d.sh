#!/bin/bash
# Round-6 end artifacts, part D: every legal average x {VM image, random} with board power and
# clock (scripts/avg_table.py), config 2 at the power cap
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/final_r06d}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step table 600 python scripts/avg_table.py || exit 1
step c2power 200 python scripts/avg_table.py --kinds random --avgs 4194304 --size-gib 8 --steps 50 --warmup 30 || exit 1
echo done
