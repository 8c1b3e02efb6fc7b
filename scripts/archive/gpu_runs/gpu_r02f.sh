#!/bin/bash
# in-house sort/scan: the paths that use them (multi-kernel resolve, candidate lists, sharded
# phases, known chunks), then the whole GPU suite
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=gpurun_out/r02f; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step sortpaths 400 python -u -m pytest tests -m gpu -k "resolve_paths or candidates or periodic or known or shard or small_batches or upload or 3GiB" -x -v --timeout 200 --timeout-method thread || exit 1
step pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread || exit 1
step c5_unfused 300 env PBS_FUSED=0 python bench.py --cpu-baseline 0 --host-inclusive-gib 0 --avg 262144 || exit 1
step b64k 300 python bench.py --cpu-baseline 0 --host-inclusive-gib 0 --avg 65536 --steps 3 || exit 1
step digest 400 python bench.py --steps 2 --warmup 1 --cpu-baseline 0 --host-inclusive-gib 0 --digest 1 || exit 1
echo done
