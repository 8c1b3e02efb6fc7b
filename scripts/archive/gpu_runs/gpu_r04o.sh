#!/bin/bash
# Round 4o: scan pass without copies after its kernel (gather results and, into a pinned cut
# array, the resolve's cuts straight to host memory): parity tests, the split, then the
# tile-end / concurrency / resolver-priority A/Bs.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r04o}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step tests 500 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -k "scan_pass or pinned or resolve_paths or small_batches or fused" || exit 1
step split 300 python scripts/scan_pass_split.py || exit 1
step split_copy 300 env PBS_DIRECT_OUT=0 python scripts/scan_pass_split.py --avgs 65536,131072 || exit 1
step tileend 400 python scripts/tile_end_ab.py || exit 1
step conc 300 python scripts/concurrent_pass_ab.py || exit 1
step ab 500 env PBS_DEBUG_PHASES=1 python scripts/resolver_prio_ab.py --prios 0,3,15,11 || exit 1
echo done
