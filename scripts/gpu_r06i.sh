#!/bin/bash
# bisect: the 64 GiB VM-image blob stage and the 1 GiB VM corpus on the builds of this round
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r06i}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
for c in d02ec6e b622fc4 9104347; do
  L=scripts/ab_libs/w_$c/proxmox-backup_amd/csrc/libpbschunk.so
  step vm_$c 200 env PBS_ZSTD_SPLIT=0 PBS_LIBPBSCHUNK_AB=$L python scripts/zstd_bench.py --corpus vm --gib 1 --reps 2 || exit 1
done
step vm_head_fused 200 env PBS_ZSTD_SPLIT=0 python scripts/zstd_bench.py --corpus vm --gib 1 --reps 2 || exit 1
step vm_head 200 python scripts/zstd_bench.py --corpus vm --gib 1 --reps 2 || exit 1
step blobs_d02ec6e 300 env PBS_LIBPBSCHUNK_AB=scripts/ab_libs/w_d02ec6e/proxmox-backup_amd/csrc/libpbschunk.so python bench.py --stages 0 --blobs 1 --steps 5 --warmup 2 || exit 1
step blobs_b622fc4 300 env PBS_LIBPBSCHUNK_AB=scripts/ab_libs/w_b622fc4/proxmox-backup_amd/csrc/libpbschunk.so python bench.py --stages 0 --blobs 1 --steps 5 --warmup 2 || exit 1
echo done
