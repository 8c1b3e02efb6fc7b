#!/bin/bash
# the VM-image corpus: phase probes (split head, fused head, fused b622fc4) and a kernel trace
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r06j}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
B=scripts/ab_libs/w_b622fc4/proxmox-backup_amd/csrc/libpbschunk.so
step probe_split 200 env PBS_ZSTD_PROBE=1 python scripts/zstd_bench.py --corpus vm --gib 1 --reps 1 || exit 1
step probe_fused 200 env PBS_ZSTD_PROBE=1 PBS_ZSTD_SPLIT=0 python scripts/zstd_bench.py --corpus vm --gib 1 --reps 1 || exit 1
step probe_b622 200 env PBS_ZSTD_PROBE=1 PBS_LIBPBSCHUNK_AB=$B python scripts/zstd_bench.py --corpus vm --gib 1 --reps 1 || exit 1
step trace_split 200 rocprofv3 --kernel-trace --stats -d $O/prof_split -o run -- python3 scripts/zstd_bench.py --corpus vm --gib 1 --reps 2 || exit 1
step trace_b622 200 env PBS_LIBPBSCHUNK_AB=$B rocprofv3 --kernel-trace --stats -d $O/prof_b622 -o run -- python3 scripts/zstd_bench.py --corpus vm --gib 1 --reps 2 || exit 1
python3 scripts/ktrace.py $(ls $O/prof_split/*/run_results.db $O/prof_split/run_results.db 2>/dev/null | head -1) zstd > $O/k_split.txt
echo done
