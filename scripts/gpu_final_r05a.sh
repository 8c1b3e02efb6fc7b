#!/bin/bash
# Round-5 end artifacts, part A: every GPU test, smoke, PMC traffic of the fused kernel on the
# VM image and on random bytes (before the bench, so the bench line carries both), the default
# bench line and rocprofv3 kernel stats of the same command.  Each GPU step has its own time
# limit; the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R="$(pwd)"; export TMPDIR=/tmp; O=${OUT:-gpurun_out/final_r05}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
NOEXTRA="--cpu-baseline 0 --cpu-config1 0 --host-inclusive-gib 0 --secondary-random 0"
step pytest_gpu 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread || exit 1
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step pmc 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/$O/pmc_fetch" -o run -- python bench.py --steps 3 --warmup 1 $NOEXTRA || exit 1
python profiles/collect_traffic.py "$O/pmc_fetch" --out "$O/traffic.json" > "$O/collect.log" 2>&1 && cp "$O/traffic.json" profiles/traffic_latest.json
step pmc_random 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/$O/pmc_fetch_random" -o run -- python bench.py --workload random --steps 3 --warmup 1 $NOEXTRA || exit 1
python profiles/collect_traffic.py "$O/pmc_fetch_random" --workload random --out "$O/traffic_random.json" > "$O/collect_random.log" 2>&1 && cp "$O/traffic_random.json" profiles/traffic_random.json
step bench64 300 python bench.py || exit 1
step rocprof 150 rocprofv3 --kernel-trace --stats -d "$R/$O/prof" -o run --output-format csv -- python bench.py --steps 5 --warmup 1 $NOEXTRA || exit 1
echo done
