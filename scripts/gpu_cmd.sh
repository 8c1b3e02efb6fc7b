set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/sha; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_digest.py tests/test_gpu_blob.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/sha/pytest.log 2>&1
echo rc=$?
