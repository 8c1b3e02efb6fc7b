#!/bin/bash
# Round 4zc: the scan pass's one host sync -- stream sync vs event sync on the last kernel
# (PBS_SYNC_MODE 0/1), alternated in one process at 64 / 128 KiB, both data kinds.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r04zc}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step ab 600 python scripts/tile_end_ab.py --env PBS_SYNC_MODE --dbg 0,1 --kinds random,vmimage --avgs 131072,65536 --steps 8 --reps 3 || exit 1
echo done
