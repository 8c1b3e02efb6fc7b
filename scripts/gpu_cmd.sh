set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 500 --timeout-method thread -k "full_size" > gpurun_out/pytest_full3.log 2>&1
echo rc=$?
