#!/bin/bash
# Round-5 end artifacts, part C: PMC per-byte records of the final build -- the headline scan
# kernel on the VM image vs random bytes (scripts/scan_pmc.sh) and the zstd block kernel on the
# text / pxar corpora, this build vs round 4's (scripts/zstd_pmc.sh) -- summarised per byte.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/final_r05}; mkdir -p $O
bash scripts/scan_pmc.sh > "$O/scan_pmc.log" 2>&1 || exit 1
python3 scripts/pmc_per_byte.py gpurun_out/pmc_scan --kernel scan_fused_kernel --bytes 68719476736 > "$O/pmc_scan_per_byte.jsonl" 2>&1 || exit 1
BUILDS="cur r04" bash scripts/zstd_pmc.sh > "$O/zstd_pmc.log" 2>&1 || exit 1
python3 scripts/pmc_per_byte.py gpurun_out/pmc_zstd --kernel zstd_block_kernel > "$O/pmc_zstd_per_byte.jsonl" 2>&1 || exit 1
echo done
