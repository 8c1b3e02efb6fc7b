set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_digest.py -m gpu -x -v --timeout 300 --timeout-method thread -k "upload or pipeline" > gpurun_out/pytest_upload.log 2>&1
echo rc=$?
