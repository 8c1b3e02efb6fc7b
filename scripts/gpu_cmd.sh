set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/fold; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 500 --timeout-method thread > gpurun_out/fold/pytest.log 2>&1 && \
timeout -k 10 400 python bench.py --steps 10 --warmup 2 --cpu-baseline 0 --host-inclusive-gib 0 > gpurun_out/fold/bench64.log 2>&1 && \
timeout -k 10 400 python bench.py --steps 10 --warmup 2 --cpu-baseline 0 --host-inclusive-gib 0 > gpurun_out/fold/bench64b.log 2>&1
echo rc=$?
