set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/examples; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_examples.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_examples.log 2>&1 && \
timeout -k 10 200 examples/test_chunk_speed > gpurun_out/examples/test_chunk_speed.txt 2>&1 && \
timeout -k 10 200 examples/test_chunk_speed2 > gpurun_out/examples/test_chunk_speed2.txt 2>&1 && \
timeout -k 10 200 examples/test_chunk_size > gpurun_out/examples/test_chunk_size.txt 2>&1
echo rc=$?
