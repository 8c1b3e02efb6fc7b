set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/pipeline; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_digest.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pipeline/pytest.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --cpu-baseline 0 --host-inclusive-gib 0 --pipeline-gib 64 > gpurun_out/pipeline/bench_pipe_crc.log 2>&1
echo rc=$?
