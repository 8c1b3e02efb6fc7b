#!/bin/bash
# Round 3: A/B across builds -- exact windows in flight at tile ends 8 (product) vs 16
# (scripts/variants/libPD16.so), alternating processes, 64 GiB VM image at 64 KiB .. 4 MiB.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r03_pd}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
for avg in 65536 262144 4194304; do
  for rep in 1 2; do
    step pd8_${avg}_$rep 300 env DIAG_CONFIGS=PBS_BALANCE=1 python scripts/pass_diag.py 64 vmimage $avg 8 || exit 1
    step pd16_${avg}_$rep 300 env DIAG_LIB=scripts/variants/libPD16.so DIAG_CONFIGS=PBS_BALANCE=1 python scripts/pass_diag.py 64 vmimage $avg 8 || exit 1
  done
done
echo done
