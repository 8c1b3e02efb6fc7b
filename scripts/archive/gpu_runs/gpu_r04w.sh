#!/bin/bash
# Round 4w: host SHA-256 with up to four chunks in step per thread (sha256_host_lanes) in the
# host-stream pipeline.  Digest tests; same-process sweep: one at a time vs lanes, routing
# variants for the faster host share; the bench's pipeline stage.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r04w}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step tests 400 python -u -m pytest tests/test_gpu_digest.py -x -v --timeout 200 --timeout-method thread || exit 1
step sweep 600 python scripts/pipe_sweep.py "PBS_SHA_HOST_LANES=1" "" "GPU_MBS=20" "SLACK_MS=0" "GPU_MBS=20,SLACK_MS=0" "GPU_MBS=15,SLACK_MS=0" "" "PBS_SHA_HOST_LANES=1" || exit 1
step bench 600 python bench.py --pipeline-gib 64 || exit 1
echo done
