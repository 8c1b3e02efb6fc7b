set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 scripts/host_bench 1 > gpurun_out/host_bench.log 2>&1 && \
PBS_STAGE_DIRECT=1 timeout -k 10 300 scripts/host_bench 1 > gpurun_out/host_bench_direct.log 2>&1
echo rc=$?
