#!/bin/bash
# scan server: per-request phases for 64 KiB / 256 KiB / 1 MiB reads, slot in VRAM vs pinned (PBS_SERVER_VRAM_MAX)
set -o pipefail
mkdir -p gpurun_out/srvp
for p in 65536 262144 1048576; do
  PBS_SERVER_PROBE=1 timeout -k 10 60 examples/test_chunk_speed2 - 1073741824 $p 4194304 0 1 > gpurun_out/srvp/p_$p.log 2>&1 || exit 1
  PBS_SERVER_VRAM_MAX=131072 PBS_SERVER_PROBE=1 timeout -k 10 60 examples/test_chunk_speed2 - 1073741824 $p 4194304 0 1 > gpurun_out/srvp/p_${p}_host.log 2>&1 || exit 1
  PBS_SERVER_VRAM_MAX=131072 timeout -k 10 60 examples/test_chunk_speed2 - 1073741824 $p 4194304 0 1 > gpurun_out/srvp/r_${p}_host.log 2>&1 || exit 1
done
