#!/bin/bash
# scan_main with per-wave LDS suspect lists: parity, zstd encoder prefetch, 64 KiB and config 2
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=gpurun_out/r02ad; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step parity 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_zstd.py -x -v --timeout 300 --timeout-method thread || exit 1
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step a64k 300 python bench.py --steps 5 --warmup 2 --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0 --avg 65536 || exit 1
step c2 300 python bench.py --steps 50 --warmup 30 --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0 --size-gib 8 --workload random || exit 1
step blobs 300 python bench.py --steps 2 --warmup 1 --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0 --blobs 1 || exit 1
echo done
