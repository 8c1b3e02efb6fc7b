#!/bin/bash
# Host SHA-256 on the GPU box's CPU: one message at a time vs 2-4 in step, and the
# multi-lane scheduler over a chunk list on 1 and 14 threads (CPU only).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04v; mkdir -p $O
g++ -O2 -std=c++17 -I proxmox-backup_amd/csrc -I include scripts/sha_host_lanes_bench.cpp -o /tmp/sha_lanes -lpthread || exit 1
grep -m1 "model name" /proc/cpuinfo > $O/sha_lanes.log
timeout -k 10 120 /tmp/sha_lanes >> $O/sha_lanes.log 2>&1 || exit 1
cat $O/sha_lanes.log
