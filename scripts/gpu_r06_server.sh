#!/bin/bash
# scan() per read through the scan server (the unchanged ChunkStream caller) at 8 / 64 /
# 256 KiB reads: PBS_SERVER_PROBE phase split, and the split-request knobs
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r06_server}; mkdir -p $O
run() { local name=$1; shift; timeout -k 10 120 env "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
for p in 8192 65536 262144; do
  run probe_$p PBS_SERVER_PROBE=1 examples/test_chunk_speed2 - 1073741824 $p 4194304 0 1 || exit 1
  run base_$p PBS_X=0 examples/test_chunk_speed2 - 1073741824 $p 4194304 0 1 || exit 1
done
for mp in 1 2 4; do
  run mp${mp}_65536 PBS_SERVER_MINPASS=$mp examples/test_chunk_speed2 - 1073741824 65536 4194304 0 1 || exit 1
  run mp${mp}_262144 PBS_SERVER_MINPASS=$mp examples/test_chunk_speed2 - 1073741824 262144 4194304 0 1 || exit 1
done
run wg32_65536 PBS_SERVER_WGS=32 PBS_SERVER_MINPASS=1 examples/test_chunk_speed2 - 1073741824 65536 4194304 0 1 || exit 1
echo done
