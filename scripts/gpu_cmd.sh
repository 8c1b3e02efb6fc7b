set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/dyn; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 500 --timeout-method thread -k "full_size" > gpurun_out/dyn/pytest_full2.log 2>&1 && \
timeout -k 10 400 python scripts/ab_dyn.py 64 4194304 1:16384:0 1:16384:1 0:32768 > gpurun_out/dyn/ab64d.log 2>&1 && \
timeout -k 10 400 python scripts/ab_dyn.py 64 262144 1:16384:0 1:16384:1 > gpurun_out/dyn/ab64d_256k.log 2>&1
echo rc=$?
