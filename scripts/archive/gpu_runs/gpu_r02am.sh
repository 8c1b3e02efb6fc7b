#!/bin/bash
# tile-order rules: 1 MiB / 256 KiB / 4 MiB at 64 GiB, 256 KiB at 8 GiB; headline bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=gpurun_out/r02am; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step fused_tests 300 python -u -m pytest tests/test_gpu_parity.py -k "fused or golden or split" -x -v --timeout 120 --timeout-method thread || exit 1
step a1m 300 env DIAG_CONFIGS="PBS_SCAN_DYN=1;PBS_SCAN_DYN=0" python scripts/pass_diag.py 64 vmimage 1048576 6 || exit 1
step c5_8 300 env DIAG_CONFIGS="PBS_FUSED=0;PBS_FUSED=1,PBS_SCAN_DYN=0" python scripts/pass_diag.py 8 vmimage 262144 30 || exit 1
step a512k 300 env DIAG_CONFIGS="PBS_SCAN_DYN=1;PBS_SCAN_DYN=0" python scripts/pass_diag.py 64 vmimage 524288 6 || exit 1
step bench64 600 python bench.py --cpu-baseline 0 --host-inclusive-gib 0 || exit 1
step c2 300 python bench.py --steps 50 --warmup 30 --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0 --size-gib 8 --workload random || exit 1
echo done
