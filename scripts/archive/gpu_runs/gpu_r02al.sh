#!/bin/bash
# resolver lag after the last tile: static+balance vs dynamic, 256 KiB and 4 MiB
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=gpurun_out/r02al; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step c5 300 env PBS_DEBUG_PHASES=1 DIAG_CONFIGS="PBS_SCAN_DYN=1;PBS_SCAN_DYN=0" python scripts/pass_diag.py 64 vmimage 262144 1 || exit 1
step c3 300 env PBS_DEBUG_PHASES=1 DIAG_CONFIGS="PBS_SCAN_DYN=1;PBS_SCAN_DYN=0" python scripts/pass_diag.py 64 vmimage 4194304 1 || exit 1
echo done
