#!/bin/bash
# Round 4p: scan-pass kernel vs candidate count: the scan pass forced at 256 KiB .. 4 MiB
# (PBS_FUSED_MIN_AVG=8M) beside the fused pass; the tile-end "no exact hash" switch at 4 MiB.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r04p}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step minavg 400 python scripts/tile_end_ab.py --kinds vmimage --avgs 262144,1048576,4194304 --env PBS_FUSED_MIN_AVG --dbg 262144,8388608 || exit 1
step dbg4m 300 python scripts/tile_end_ab.py --kinds vmimage --avgs 4194304 --env PBS_FUSED_MIN_AVG --dbg 8388608 --reps 1 || exit 1
step dbg4m1 300 env PBS_FUSED_DBG=1 python scripts/tile_end_ab.py --kinds vmimage --avgs 4194304 --env PBS_FUSED_MIN_AVG --dbg 8388608 --reps 1 || exit 1
echo done
