#!/bin/bash
# PMC passes over single microbench variants (separate --pmc runs, kernel-trace only)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT="$(pwd)/gpurun_out/pmc"
mkdir -p "$OUT"
rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
for v in ${VARIANTS:-0 2 3}; do
  for ctr in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
             "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS" \
             "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_MISC" \
             "FETCH_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
    tag=$(echo $ctr | tr ' ' '_' | cut -c1-40)
    timeout -k 10 120 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/v${v}_$tag" -o run -- scripts/microbench/mb_scan 16 2 $v > "$OUT/v${v}_$tag.log" 2>&1
    rc=$?; echo "variant $v [$ctr] rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
done
