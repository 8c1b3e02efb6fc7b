set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_digest.py -m gpu -x -q --timeout 300 -k pipeline > gpurun_out/pytest_pipe.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --cpu-baseline 0 --host-inclusive-gib 0 --pipeline-gib 64 > gpurun_out/bench_pipe.log 2>&1
echo rc=$?
