#!/bin/bash
# Round 4b: fused pass vs scan pass at 256 KiB / 512 KiB (random and VM image), same process.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r04b}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step r256 300 python scripts/ab_handles.py random 64 262144 fused scan:PBS_FUSED_MIN_AVG=524288 || exit 1
step v256 300 python scripts/ab_handles.py vmimage 64 262144 fused scan:PBS_FUSED_MIN_AVG=524288 || exit 1
step r512 300 python scripts/ab_handles.py random 64 524288 fused scan:PBS_FUSED_MIN_AVG=1048576 || exit 1
step r64 300 python scripts/ab_handles.py random 64 65536 scan multi:PBS_SCAN_PASS=0 || exit 1
echo done
