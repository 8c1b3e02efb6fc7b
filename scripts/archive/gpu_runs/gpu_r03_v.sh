#!/bin/bash
# Round 3: validation of the scan pass (64 KiB averages) and the scan-server ack shortcut:
# the full GPU suite, smoke, the unchanged caller's 8 KiB / 256 KiB reads, 64 KiB and the
# headline bench (same box).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r03_v}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || exit 1
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step ex_8k 120 examples/test_chunk_speed2 - 1073741824 8192 4194304 0 1 || exit 1
step ex_8k_b 120 examples/test_chunk_speed2 - 1073741824 8192 4194304 0 1 || exit 1
step ex_8k_probe 120 env PBS_SERVER_PROBE=1 examples/test_chunk_speed2 - 1073741824 8192 4194304 0 1 || exit 1
step ex_256k 120 examples/test_chunk_speed2 - 1073741824 262144 4194304 0 1 || exit 1
step a64k 300 python bench.py --steps 5 --warmup 2 --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0 --avg 65536 || exit 1
step a64k_old 300 env PBS_SCAN_PASS=0 python bench.py --steps 5 --warmup 2 --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0 --avg 65536 || exit 1
step bench64 300 python bench.py --steps 10 --warmup 3 --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0 || exit 1
echo done
