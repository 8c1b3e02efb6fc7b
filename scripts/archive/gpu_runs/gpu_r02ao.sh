#!/bin/bash
# balancing mode 3 (the wave ahead waits for its partner): probe pair gaps + A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=gpurun_out/r02ao; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
for b in 1 3; do step probe_c2_b$b 200 env PBS_BALANCE=$b python scripts/microbench/fused_probe.py 8 random 4194304 || exit 1; done
step c2 300 env DIAG_CONFIGS="PBS_BALANCE=0;PBS_BALANCE=1;PBS_BALANCE=3" python scripts/pass_diag.py 8 random 4194304 30 || exit 1
step c3 300 env DIAG_CONFIGS="PBS_BALANCE=0;PBS_BALANCE=1;PBS_BALANCE=3" python scripts/pass_diag.py 64 vmimage 4194304 6 || exit 1
echo done
