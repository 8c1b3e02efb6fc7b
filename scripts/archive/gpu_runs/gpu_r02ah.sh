#!/bin/bash
# per-wave timeline of the fused kernel (probe build): 8 GiB static / dynamic, 64 GiB; fused dynamic at 8 GiB
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=gpurun_out/r02ah; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step probe_c2 300 python scripts/microbench/fused_probe.py 8 random 4194304 || exit 1
step probe_c2_dyn 300 env PBS_SCAN_DYN=1 python scripts/microbench/fused_probe.py 8 random 4194304 || exit 1
step probe_64 300 python scripts/microbench/fused_probe.py 64 vmimage 4194304 || exit 1
step diag_c2_dyn 300 env PBS_SCAN_DYN=1 python scripts/pass_diag.py 8 random 4194304 50 || exit 1
echo done
