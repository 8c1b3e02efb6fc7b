#!/bin/bash
# Pass time split multi-launch vs fused (config 2, 64 KiB), effective shader clock of the
# headline kernel on the VM image and on random data (GRBM_GUI_ACTIVE pass).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R="$(pwd)"; export TMPDIR=/tmp; O=gpurun_out/r02ae; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step diag_c2 300 python scripts/pass_diag.py 8 random 4194304 50 || exit 1
step diag_64k 300 env DIAG_MODES=0 python scripts/pass_diag.py 64 vmimage 65536 5 || exit 1
step clk_vm 120 rocprofv3 --pmc GRBM_GUI_ACTIVE --output-format csv -d "$R/$O/clk_vm" -o run -- python bench.py --steps 3 --warmup 2 --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0 || exit 1
step clk_rand 120 rocprofv3 --pmc GRBM_GUI_ACTIVE --output-format csv -d "$R/$O/clk_rand" -o run -- python bench.py --steps 3 --warmup 2 --cpu-baseline 0 --host-inclusive-gib 0 --secondary-random 0 --workload random || exit 1
echo done
