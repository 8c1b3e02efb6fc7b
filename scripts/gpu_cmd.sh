set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
# 101 stream_read nt, 100 stream_read, 9 v3 loads-only (8 waves), 1 FR2 full
for v in 101 100 9 1; do
  timeout -k 10 60 scripts/microbench/mb_scan 32 600 $v 1 > gpurun_out/pw_v$v.log 2>&1 &
  pid=$!
  sleep 1.0
  for k in 1 2 3 4 5 6; do amd-smi metric -p -c -g 0 >> gpurun_out/pw_v$v.log 2>&1; sleep 0.2; done
  wait $pid || exit 1
done
echo ok
