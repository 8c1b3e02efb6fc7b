set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 150 scripts/microbench/mb_scan 32 5 -1 0 > gpurun_out/mb_g_random.log 2>&1 && \
timeout -k 10 150 scripts/microbench/mb_scan 32 5 -1 1 > gpurun_out/mb_g_vm.log 2>&1
echo rc=$?
