#!/bin/bash
# Round 3: the fused pass's workgroup 0 dedicated to the resolver (default) vs its other three
# waves scanning (PBS_RESOLVER_WG=0), same process (pass_diag alternates); the parity tests.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=${OUT:-gpurun_out/r03_rwg}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step pytest_parity 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_concurrency.py -m gpu -x -v --timeout 300 --timeout-method thread || exit 1
step vm256k 400 env DIAG_CONFIGS="PBS_RESOLVER_WG=0;PBS_RESOLVER_WG=1" python scripts/pass_diag.py 64 vmimage 262144 8 || exit 1
step vm4m 400 env DIAG_CONFIGS="PBS_RESOLVER_WG=0;PBS_RESOLVER_WG=1" python scripts/pass_diag.py 64 vmimage 4194304 8 || exit 1
step rnd8g 300 env DIAG_CONFIGS="PBS_RESOLVER_WG=0;PBS_RESOLVER_WG=1" python scripts/pass_diag.py 8 random 4194304 30 || exit 1
echo done
