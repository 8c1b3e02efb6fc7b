#!/bin/bash
# the N > 1 path rehearsed on one GPU: two rank processes sharing it (gloo), every rank's cuts verified
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r06ab}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step n2 300 env PBS_BENCH_SHARE_GPU=1 python bench.py --gpus 2 --steps 3 --warmup 1 || exit 1
echo done
