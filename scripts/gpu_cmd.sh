set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_digest.py -m gpu -x -q --timeout 300 > gpurun_out/pytest_digest.log 2>&1
echo rc=$?
