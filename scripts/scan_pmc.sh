#!/bin/bash
# PMC passes over the headline scan kernel (scan_fused_kernel) on the 64 GiB VM image and
# on 64 GiB of random bytes: instructions and cycles per byte, the
# clock (GRBM_GUI_ACTIVE), and HBM bytes (FETCH_SIZE) for each stream.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT="$(pwd)/gpurun_out/pmc_scan"
mkdir -p "$OUT"
for wl in vmimage random; do
  for ctr in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
             "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM" \
             "GRBM_GUI_ACTIVE GRBM_COUNT" "FETCH_SIZE"; do
    tag=$(echo $ctr | cut -d' ' -f1)
    timeout -k 10 200 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/${wl}_$tag" -o run -- \
        python3 bench.py --workload $wl --steps 3 --warmup 1 --cpu-baseline 0 --cpu-config1 0 \
        --host-inclusive-gib 0 --secondary-random 0 --stages 0 > "$OUT/${wl}_$tag.log" 2>&1
    rc=$?; echo "$wl [$ctr] rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
done
