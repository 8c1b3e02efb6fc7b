#!/bin/bash
# Round 4n: tile-end A/B (scan pass 64/128 KiB), resolver issue priority A/B, a fused pass
# beside another thread's blob encoding (work areas kept vs freed every call).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r04n}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step tileend 400 python scripts/tile_end_ab.py || exit 1
step conc 300 python scripts/concurrent_pass_ab.py || exit 1
step ab 500 env PBS_DEBUG_PHASES=1 python scripts/resolver_prio_ab.py --prios 0,3,15,11 || exit 1
echo done
