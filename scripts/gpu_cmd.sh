set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/cfg; export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 50 --warmup 30 --cpu-baseline 0 --host-inclusive-gib 0 --size-gib 8 --workload random > gpurun_out/cfg/c2.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-baseline 0 --host-inclusive-gib 0 --avg 262144 > gpurun_out/cfg/c5.log 2>&1
echo rc=$?
