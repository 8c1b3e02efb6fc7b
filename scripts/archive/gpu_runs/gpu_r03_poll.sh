#!/bin/bash
# scan server with the request in VRAM: one poller (default) vs lane 0 of every wave
# polling, staggered (PBS_SERVER_POLL=4), 8 KiB test_chunk_speed2 reads, alternating.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=${OUT:-gpurun_out/poll}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
make -s -C examples || exit 1
for k in 1 2 3; do
  step ex_8k_poll1_$k 120 examples/test_chunk_speed2 - 1073741824 8192 4194304 0 1 || exit 1
  step ex_8k_poll4_$k 120 env PBS_SERVER_POLL=4 examples/test_chunk_speed2 - 1073741824 8192 4194304 0 1 || exit 1
done
step ex_8k_probe_poll4 120 env PBS_SERVER_POLL=4 PBS_SERVER_PROBE=1 examples/test_chunk_speed2 - 1073741824 8192 4194304 0 1 || exit 1
step ex_8k_probe_poll1 120 env PBS_SERVER_PROBE=1 examples/test_chunk_speed2 - 1073741824 8192 4194304 0 1 || exit 1
echo done
