#!/bin/bash
# Round 4c: the whole GPU suite after the per-device work areas (blob / digest / CRC /
# known-chunk entry points) and the bench verification.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r04c}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step conc 300 python -u -m pytest tests/test_gpu_concurrency.py -x -v --timeout 200 --timeout-method thread || exit 1
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || exit 1
step r256_8 200 python scripts/ab_handles.py random 8 262144 fused scan:PBS_FUSED_MIN_AVG=524288 || exit 1
step v256_16 200 python scripts/ab_handles.py vmimage 16 262144 fused scan:PBS_FUSED_MIN_AVG=524288 || exit 1
step r4m_64 200 python scripts/ab_handles.py random 64 4194304 fused scan:PBS_FUSED_MIN_AVG=8388608 || exit 1
echo done
