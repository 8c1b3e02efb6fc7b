#!/bin/bash
# Round 4i: pipeline routing sweep (GPU lane rate, slack) over one 64 GiB host copy.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r04i}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step sweep2 600 python scripts/pipe_sweep.py SLACK_MS=40 GPU_MBS=30,SLACK_MS=20 GPU_MBS=25,SLACK_MS=20 GPU_MBS=25,SLACK_MS=0 GPU_MBS=20,SLACK_MS=0 GPU_MBS=20,SLACK_MS=30 GPU_MBS=25,SLACK_MS=0,HOST_THREADS=15 HOST_MIN=8388608 || exit 1
echo done
