set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_digest.py -m gpu -x -q --timeout 300 > gpurun_out/pytest_digest.log 2>&1 && \
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --cpu-baseline 0 --host-inclusive-gib 0 --digest 1 > gpurun_out/bench_digest.log 2>&1 && \
PBS_SHA_ONE_WAVE=1 timeout -k 10 400 python bench.py --steps 3 --warmup 1 --cpu-baseline 0 --host-inclusive-gib 0 --digest 1 > gpurun_out/bench_digest1.log 2>&1
echo rc=$?
