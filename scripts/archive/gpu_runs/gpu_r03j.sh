#!/bin/bash
# Round 3j: zstd block kernel counters on VM-image data (I-cache, LDS, wait cycles).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=gpurun_out/r03j; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
B="python3 scripts/zstd_bench.py --corpus vm --gib 0.25 --reps 1"
step pytest_zstd 400 python -u -m pytest tests/test_gpu_zstd.py -m gpu -x -v --timeout 300 --timeout-method thread || exit 1
step corpus_probe 400 env PBS_ZSTD_PROBE=1 python3 scripts/zstd_bench.py --corpus text,pxar,vm --gib 1 --reps 2 || exit 1
step pmc_icache 180 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE --kernel-trace --output-format csv -d $O/pmc_icache -o run -- $B || exit 1
step pmc_sq 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_VALU --kernel-trace --output-format csv -d $O/pmc_sq -o run -- $B || exit 1
step pmc_sq2 180 rocprofv3 --pmc SQ_IFETCH SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_IFETCH_LEVEL --kernel-trace --output-format csv -d $O/pmc_sq2 -o run -- $B || exit 1
echo done
