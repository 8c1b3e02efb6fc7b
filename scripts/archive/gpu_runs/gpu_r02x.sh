#!/bin/bash
# fused vs multi-launch pass by stream size (config 2 = 8 GiB random)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=gpurun_out/r02x; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
for sz in 8 16 32; do
  for f in 1; do
    step s${sz}_f${f} 300 env PBS_FUSED=$f python bench.py --steps 30 --warmup 20 --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0 --size-gib $sz --workload random || exit 1
  done
done
step fused_tests 400 python -u -m pytest tests/test_gpu_parity.py -k "fused" -x -v --timeout 200 --timeout-method thread || exit 1
step s8_auto 300 python bench.py --steps 30 --warmup 20 --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0 --size-gib 8 --workload random || exit 1
echo done
