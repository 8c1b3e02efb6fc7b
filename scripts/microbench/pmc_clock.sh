#!/bin/bash
# Effective shader clock (GRBM_GUI_ACTIVE / 8 XCDs / kernel time) per microbench variant.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT="$(pwd)/gpurun_out/pmcclk"; mkdir -p "$OUT"
for v in ${VARIANTS:-0 1 2}; do
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d "$OUT/v$v" -o run -- scripts/microbench/mb_scan 32 3 $v > "$OUT/v$v.log" 2>&1
  rc=$?; echo "variant $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
