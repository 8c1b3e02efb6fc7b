#!/bin/bash
# Round 4e: H2D rates (pageable / registered / pinned), registration cost and host SHA-256
# rates -- the inputs of the host-stream pipeline model (scripts/pipe_sim.py); the
# pipeline stage as it is now.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r04e}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step h2d 300 python scripts/h2d_probe.py --gib 8 || exit 1
step pipe 400 python bench.py --steps 2 --warmup 1 --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0 --pipeline-gib 64 --verify 1 || exit 1
echo done
