#!/bin/bash
# Round 4l: pipeline work area holding the chunker, streams, events and job array between
# calls; main + copy threads hash in the drain.  Digest tests, sweeps at 1 GiB and 256 MiB
# pieces, the bench's pipeline stage.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r04l}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step tests 400 python -u -m pytest tests/test_gpu_digest.py tests/test_gpu_concurrency.py -x -v --timeout 200 --timeout-method thread || exit 1
step sweep1g 600 python scripts/pipe_sweep.py "" "" "" || exit 1
step sweep256 600 python scripts/pipe_sweep.py --piece-mib 256 "" "" "" || exit 1
step bench 600 python bench.py --pipeline-gib 64 || exit 1
echo done
