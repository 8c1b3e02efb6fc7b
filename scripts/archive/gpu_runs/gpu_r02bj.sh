#!/bin/bash
# Rehearsal of the N-rank bench path on the one-GPU box (PBS_BENCH_SHARE_GPU=1: every rank
# on GPU 0, gloo instead of RCCL; not a scaling measurement), then the round-end artifacts.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=gpurun_out/r02bj; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
PBS_BENCH_SHARE_GPU=1 step share2 300 python bench.py --gpus 2 --size-gib 16 --steps 5 --warmup 2 || exit 1
PBS_BENCH_SHARE_GPU=1 step share4 300 python bench.py --gpus 4 --size-gib 8 --steps 5 --warmup 2 || exit 1
step bench16 300 python bench.py --size-gib 16 --steps 5 --warmup 2 --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0 || exit 1
OUT=gpurun_out/final_r02i bash scripts/gpu_final_r02.sh
