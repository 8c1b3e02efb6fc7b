set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_host_mirror_cpp.py tests/test_examples.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_mirror.log 2>&1
echo rc=$?
