set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for k in 1 2 3; do timeout -k 10 120 scripts/microbench/mb_scan 32 5 -1 1 > gpurun_out/mb_seg_$k.log 2>&1 || exit 1; done
echo ok
