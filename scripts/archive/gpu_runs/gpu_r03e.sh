#!/bin/bash
# Round 3e = 3d (scan server v2) then 3c (mailbox variants, zstd throughput).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r03e bash scripts/gpu_runs/gpu_r03d.sh || exit 1
OUT=gpurun_out/r03e bash scripts/gpu_runs/gpu_r03c.sh || exit 1
