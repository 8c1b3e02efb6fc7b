#!/bin/bash
# Round 4z: the hybrid digest's host share from HBM through a pinned ring of whole-chunk
# slots (one copy stream, four chunks in step per host thread): digest tests, the bench's
# digest stage (GPU-only vs hybrid), and the ring vs the per-thread slices.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r04z}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step tests 400 python -u -m pytest tests/test_gpu_digest.py -x -v --timeout 200 --timeout-method thread || exit 1
step digest 400 python bench.py --steps 3 --warmup 1 --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0 --digest 1 || exit 1
PBS_DIGEST_RING=0 step digest_slices 400 python bench.py --steps 3 --warmup 1 --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0 --digest 1 || exit 1
echo done
