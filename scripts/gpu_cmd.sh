set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/blob; export TMPDIR=/tmp
timeout -k 10 500 python bench.py --steps 2 --warmup 1 --cpu-baseline 0 --host-inclusive-gib 0 --digest 1 > gpurun_out/blob/bench_digest.log 2>&1
echo rc=$?
