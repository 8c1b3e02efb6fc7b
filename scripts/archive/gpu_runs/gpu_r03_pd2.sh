#!/bin/bash
# Round 3: exact windows in flight 16 (product) vs 24 (scripts/variants/libPD24.so), alternating
# processes; then the fused-pass parity tests of the product build.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r03_pd2}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step pytest_parity 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread || exit 1
for avg in 65536 4194304; do
  for rep in 1 2; do
    step pd16_${avg}_$rep 300 env DIAG_CONFIGS=PBS_BALANCE=1 python scripts/pass_diag.py 64 vmimage $avg 8 || exit 1
    step pd24_${avg}_$rep 300 env DIAG_LIB=scripts/variants/libPD24.so DIAG_CONFIGS=PBS_BALANCE=1 python scripts/pass_diag.py 64 vmimage $avg 8 || exit 1
  done
done
echo done
