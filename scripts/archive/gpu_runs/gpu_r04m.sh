#!/bin/bash
# Round 4m: kernel trace of the scan pass at 64 / 128 KiB (where the ~0.3 ms after the scan
# kernel goes: gather, resolve kernels, copies).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r04m}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step trace 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/prof -o run -- python3 scripts/scan_pass_split.py --kinds random --avgs 65536,131072 --steps 4 || exit 1
echo done
