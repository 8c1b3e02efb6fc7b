#!/bin/bash
# Round-5 end artifacts, part D: configs 2 and 5, the table of every legal average x {VM image,
# random} with board power, config 2 at the power cap, and where the small-average scan pass
# spends its time beyond the kernel.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R="$(pwd)"; export TMPDIR=/tmp; O=${OUT:-gpurun_out/final_r05}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
NOEXTRA="--cpu-baseline 0 --cpu-config1 0 --host-inclusive-gib 0 --secondary-random 0"
step c2 200 python bench.py --steps 50 --warmup 30 $NOEXTRA --size-gib 8 --workload random || exit 1
step c5 200 python bench.py --steps 10 --warmup 3 $NOEXTRA --avg 262144 || exit 1
step table 500 python scripts/avg_table.py || exit 1
step c2power 200 python scripts/avg_table.py --kinds random --avgs 4194304 --size-gib 8 --steps 50 --warmup 30 || exit 1
step scan_pass_split 200 python scripts/scan_pass_split.py --kinds vmimage,random --avgs 65536,131072,262144 --steps 8 || exit 1
echo done
