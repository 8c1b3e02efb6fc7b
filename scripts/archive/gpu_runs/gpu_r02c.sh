#!/bin/bash
# fused pass v2 (batched resolver): parity subset, then bench with resolver timing
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=gpurun_out/r02c; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step fused 300 python -u -m pytest tests/test_gpu_parity.py -k "fused or golden or split or device or small or full_size" -x -v --timeout 300 --timeout-method thread || exit 1
step bench64 300 env PBS_DEBUG_PHASES=1 python bench.py --cpu-baseline 0 --host-inclusive-gib 0 || exit 1
step c5 300 env PBS_DEBUG_PHASES=1 python bench.py --cpu-baseline 0 --host-inclusive-gib 0 --avg 262144 --steps 3 || exit 1
step c5_unfused 300 env PBS_FUSED=0 python bench.py --cpu-baseline 0 --host-inclusive-gib 0 --avg 262144 || exit 1
step bench64_1M 300 env PBS_DEBUG_PHASES=1 python bench.py --cpu-baseline 0 --host-inclusive-gib 0 --avg 1048576 --steps 3 || exit 1
echo done
