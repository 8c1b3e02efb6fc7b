#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel trace only) over the zstd kernels
# (round 6: zstd_parse_kernel and zstd_entropy_kernel; PBS_ZSTD_SPLIT=0: zstd_block_kernel):
# the current build and, with BUILDS="cur r04", round 4's through PBS_LIBPBSCHUNK_AB.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT="$(pwd)/gpurun_out/pmc_zstd"
mkdir -p "$OUT"
for build in ${BUILDS:-cur}; do
  if [ "$build" = r04 ]; then export PBS_LIBPBSCHUNK_AB="$(pwd)/profiles/r05/pmc_zstd/libpbschunk_r04.so"; else unset PBS_LIBPBSCHUNK_AB; fi
  for corpus in ${CORPORA:-text pxar}; do
    for ctr in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
               "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SALU" \
               "GRBM_GUI_ACTIVE GRBM_COUNT"; do
      tag=$(echo $ctr | cut -d' ' -f1)
      timeout -k 10 150 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/${build}_${corpus}_$tag" -o run -- \
          python3 scripts/zstd_pmc_run.py --corpus $corpus > "$OUT/${build}_${corpus}_$tag.log" 2>&1
      rc=$?; echo "$build $corpus [$ctr] rc=$rc"
      [ $rc -eq 0 ] || exit $rc
    done
  done
done
