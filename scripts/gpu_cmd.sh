set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-baseline 0 --host-inclusive-gib 0 > gpurun_out/bench64.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --cpu-baseline 0 --host-inclusive-gib 0 --avg 262144 > gpurun_out/bench_c5.log 2>&1
echo rc=$?
