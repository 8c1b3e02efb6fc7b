set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_host_mirror_cpp.py -m gpu -x -q --timeout 300 > gpurun_out/pytest_mirror.log 2>&1
echo rc=$?
