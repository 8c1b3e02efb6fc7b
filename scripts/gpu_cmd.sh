set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/pipeprof; export TMPDIR=/tmp
timeout -s KILL 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pipeprof/p -o run -- python bench.py --steps 1 --warmup 0 --cpu-baseline 0 --host-inclusive-gib 0 --pipeline-gib 64 > gpurun_out/pipeprof/bench.log 2>&1
echo rc=$?
