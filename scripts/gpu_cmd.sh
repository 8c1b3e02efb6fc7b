set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_blob.py tests/test_gpu_digest.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_crc2.log 2>&1 && \
timeout -k 10 300 python scripts/ab_crc.py > gpurun_out/ab_crc2.log 2>&1
echo rc=$?
