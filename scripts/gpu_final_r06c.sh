#!/bin/bash
# Round-6 end artifacts, part C: PMC per-byte records -- the headline scan kernel on the VM
# image and random bytes (scripts/scan_pmc.sh), the zstd parse and entropy kernels on the
# text / pxar corpora (scripts/zstd_pmc.sh) -- summarised per input byte.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/final_r06}; mkdir -p $O
bash scripts/scan_pmc.sh > "$O/scan_pmc.log" 2>&1 || exit 1
python3 scripts/pmc_per_byte.py gpurun_out/pmc_scan --kernel scan_fused_kernel --bytes 68719476736 > "$O/pmc_scan_per_byte.jsonl" 2>&1 || exit 1
BUILDS=cur bash scripts/zstd_pmc.sh > "$O/zstd_pmc.log" 2>&1 || exit 1
python3 scripts/pmc_per_byte.py gpurun_out/pmc_zstd --kernel zstd_parse_kernel > "$O/pmc_zstd_parse_per_byte.jsonl" 2>&1 || exit 1
python3 scripts/pmc_per_byte.py gpurun_out/pmc_zstd --kernel zstd_entropy_kernel > "$O/pmc_zstd_entropy_per_byte.jsonl" 2>&1 || exit 1
echo done
