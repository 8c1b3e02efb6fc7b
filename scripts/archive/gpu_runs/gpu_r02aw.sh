#!/bin/bash
# where the static order loses at small averages: scanner finish vs kernel end (probe build)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=gpurun_out/r02aw; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
for d in 0 1; do
  step p128_d$d 200 env PBS_SCAN_DYN=$d PBS_DEBUG_PHASES=1 python scripts/microbench/fused_probe.py 64 vmimage 131072 || exit 1
  step p4m_d$d 200 env PBS_SCAN_DYN=$d PBS_DEBUG_PHASES=1 python scripts/microbench/fused_probe.py 64 vmimage 4194304 || exit 1
done
echo done
