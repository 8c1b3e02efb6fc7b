#!/bin/bash
# Round 4x: routing sweep for the pipeline with the four-lane host SHA-256 (the host share
# can now take more of the late chunks: lower assumed GPU lane rate, less slack).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r04x}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step sweep 700 python scripts/pipe_sweep.py "GPU_MBS=15,SLACK_MS=0" "GPU_MBS=12,SLACK_MS=0" "GPU_MBS=10,SLACK_MS=0" "GPU_MBS=15,SLACK_MS=10" "GPU_MBS=17,SLACK_MS=0" "GPU_MBS=12,SLACK_MS=10" "GPU_MBS=15,SLACK_MS=0,HOST_THREADS=15" "GPU_MBS=15,SLACK_MS=0" "GPU_MBS=12,SLACK_MS=0" || exit 1
echo done
