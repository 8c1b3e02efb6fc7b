#!/bin/bash
# bench.py's timed passes with the cut list DMA'd into a pinned host array (--pinned-out 1,
# the default now) vs a pageable array per call (0): 64 KiB and 256 KiB averages and the
# 4 MiB headline, alternating in one box.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=${OUT:-gpurun_out/pinout}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
B="python bench.py --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0"
step pytest 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 120 --timeout-method thread -k "find_cuts_device" || exit 1
for k in 1 2; do
  for p in 1 0; do
    step a64k_p${p}_$k 300 $B --steps 5 --warmup 2 --avg 65536 --pinned-out $p || exit 1
  done
done
for p in 1 0; do
  step c5_p$p 300 $B --steps 10 --warmup 3 --avg 262144 --pinned-out $p || exit 1
  step h4m_p$p 300 $B --steps 10 --warmup 3 --pinned-out $p || exit 1
done
echo done
