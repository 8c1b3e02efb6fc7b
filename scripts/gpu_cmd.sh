set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/dyn; export TMPDIR=/tmp
timeout -k 10 300 python scripts/ab_dyn.py 8 4194304 0:32768 1:16384:1 1:8192:1 > gpurun_out/dyn/ab8e.log 2>&1 && \
timeout -k 10 300 python scripts/ab_dyn.py 16 4194304 0:32768 1:16384:1 1:8192:1 > gpurun_out/dyn/ab16e.log 2>&1 && \
timeout -k 10 300 python scripts/ab_dyn.py 32 4194304 0:32768 1:16384:1 1:8192:1 > gpurun_out/dyn/ab32e.log 2>&1 && \
timeout -k 10 300 python scripts/ab_dyn.py 2 4194304 0:32768 1:16384:1 1:8192:1 > gpurun_out/dyn/ab2e.log 2>&1
echo rc=$?
