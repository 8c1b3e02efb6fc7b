#!/bin/bash
# Round-6 end artifacts, part A: every GPU test, smoke, the PMC traffic records of the fused
# scan kernel on the VM image and on random bytes (before the bench, so the line carries
# both), the default bench line under a rocprofv3 kernel trace (the SAME process: the trace
# recomputes the line's frac, scripts/frac_from_trace.py), and the default line unprofiled.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R="$(pwd)"; export TMPDIR=/tmp; O=${OUT:-gpurun_out/final_r06}; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
NOEXTRA="--cpu-baseline 0 --cpu-config1 0 --host-inclusive-gib 0 --secondary-random 0 --stages 0"
step pytest_gpu 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread || exit 1
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step pmc 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/$O/pmc_fetch" -o run -- python bench.py --steps 3 --warmup 1 $NOEXTRA || exit 1
python profiles/collect_traffic.py "$O/pmc_fetch" --out "$O/traffic.json" > "$O/collect.log" 2>&1 && cp "$O/traffic.json" profiles/traffic_latest.json
step pmc_random 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/$O/pmc_fetch_random" -o run -- python bench.py --workload random --steps 3 --warmup 1 $NOEXTRA || exit 1
python profiles/collect_traffic.py "$O/pmc_fetch_random" --workload random --out "$O/traffic_random.json" > "$O/collect_random.log" 2>&1 && cp "$O/traffic_random.json" profiles/traffic_random.json
step bench_traced 400 rocprofv3 --kernel-trace --stats --output-format csv rocpd -d "$R/$O/prof" -o run -- python bench.py || exit 1
python scripts/frac_from_trace.py "$O/prof" --bench "$O/bench_traced.log" > "$O/frac_from_trace.json" 2>&1
step bench 400 python bench.py || exit 1
echo done
