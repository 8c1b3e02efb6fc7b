#!/bin/bash
# Round 4z3: the hybrid digest's ring with one vs two D2H copy streams (same process
# order alternated by separate bench runs).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r04z3}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
B="python bench.py --steps 3 --warmup 1 --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0 --digest 1"
step one_a 300 $B || exit 1
PBS_DIGEST_RING_STREAMS=2 step two_a 300 $B || exit 1
step one_b 300 $B || exit 1
PBS_DIGEST_RING_STREAMS=2 step two_b 300 $B || exit 1
echo done
