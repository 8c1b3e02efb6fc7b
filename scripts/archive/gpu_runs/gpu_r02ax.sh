#!/bin/bash
# probe build without spills: per-wave timelines, static order with / without balancing
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=gpurun_out/r02ax; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
for b in 0 1; do
  step p8_b$b 200 env PBS_BALANCE=$b python scripts/microbench/fused_probe.py 8 random 4194304 || exit 1
  step p64_b$b 200 env PBS_BALANCE=$b python scripts/microbench/fused_probe.py 64 vmimage 4194304 || exit 1
done
step p64_dyn 200 env PBS_SCAN_DYN=1 python scripts/microbench/fused_probe.py 64 vmimage 4194304 || exit 1
echo done
