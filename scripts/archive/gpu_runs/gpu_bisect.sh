#!/bin/bash
# Bisect a parity failure over prebuilt library variants (scripts/variants/lib*.so).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=gpurun_out/bisect; mkdir -p $O
cp proxmox-backup_amd/csrc/libpbschunk.so /tmp/lib_orig.so
for v in ${VARIANTS:-A B C}; do
  cp scripts/variants/lib$v.so proxmox-backup_amd/csrc/libpbschunk.so
  timeout -k 10 200 python -u -m pytest tests/test_gpu_zstd.py -m gpu -x -q --timeout 150 --timeout-method thread > $O/$v.log 2>&1
  rc=$?; echo "variant $v rc=$rc"
  if [ $rc -ge 124 ]; then break; fi
done
cp /tmp/lib_orig.so proxmox-backup_amd/csrc/libpbschunk.so
