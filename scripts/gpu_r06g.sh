#!/bin/bash
# scan server: followers poll the host record; one pass per workgroup
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r06g}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
step tests 400 $PYT -m gpu tests/test_gpu_parity.py -k "server or scan_call or stream or chunker1" tests/test_examples.py tests/test_shim_sequence.py tests/test_host_mirror_cpp.py || exit 1
for r in 1 2; do
for p in 8192 16384 65536 262144 1048576; do
  step ex_${p}_$r 120 examples/test_chunk_speed2 - 1073741824 $p 4194304 0 1 || exit 1
done
done
step probe_65536 120 env PBS_SERVER_PROBE=1 examples/test_chunk_speed2 - 1073741824 65536 4194304 0 1 || exit 1
step probe_8192 120 env PBS_SERVER_PROBE=1 examples/test_chunk_speed2 - 1073741824 8192 4194304 0 1 || exit 1
echo done
