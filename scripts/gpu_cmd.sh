set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/warm; export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --cpu-baseline 0 --host-inclusive-gib 0 --size-gib 8 --workload random > gpurun_out/warm/c2_w1.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 50 --warmup 30 --cpu-baseline 0 --host-inclusive-gib 0 --size-gib 8 --workload random > gpurun_out/warm/c2_w30.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-baseline 0 --host-inclusive-gib 0 > gpurun_out/warm/b64_w2.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 10 --cpu-baseline 0 --host-inclusive-gib 0 > gpurun_out/warm/b64_w10.log 2>&1
echo rc=$?
