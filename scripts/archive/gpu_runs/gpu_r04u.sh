#!/bin/bash
# Round 4u: pipeline -- small tail pieces (PBS_PIPE_TAIL_MIB / TAIL_PIECE_MIB) and piecewise
# registration of the host buffer (PBS_PIPE_REGISTER) over one page-aligned 64 GiB copy,
# settings alternated in one process; the digest tests with both on.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r04u}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step tests_skip 1 true || true
: step tests 400 env PBS_PIPE_REGISTER=1 PBS_PIPE_TAIL_MIB=24 PBS_PIPE_TAIL_PIECE_MIB=3 python -u -m pytest tests/test_gpu_digest.py -x -v --timeout 200 --timeout-method thread -k pipeline || exit 1
step sweep 700 python scripts/pipe_sweep.py --aligned "" "REGISTER=1" "TAIL_MIB=4096,TAIL_PIECE_MIB=256" "REGISTER=1,TAIL_MIB=4096,TAIL_PIECE_MIB=256" "" "REGISTER=1" "TAIL_MIB=4096,TAIL_PIECE_MIB=256" "REGISTER=1,TAIL_MIB=4096,TAIL_PIECE_MIB=256" || exit 1
echo done
