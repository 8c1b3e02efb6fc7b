#!/bin/bash
# scan server split over workgroups: parity tests, then 256 KiB / 8 KiB / 1 MiB reads per workgroup count
set -o pipefail
mkdir -p gpurun_out/srv
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_concurrency.py -m gpu -k "scan_server or scan_feed or beside_scan_server or chunker1" > gpurun_out/srv/tests.log 2>&1 || exit 1
for w in 1 4 8 16 32; do
  PBS_SERVER_WGS=$w timeout -k 10 60 examples/test_chunk_speed2 - 1073741824 262144 4194304 0 1 > gpurun_out/srv/ex256_w$w.log 2>&1 || exit 1
done
PBS_SERVER_PROBE=1 timeout -k 10 60 examples/test_chunk_speed2 - 1073741824 262144 4194304 0 1 > gpurun_out/srv/ex256_probe.log 2>&1 || exit 1
for p in 8192 65536 1048576; do
  timeout -k 10 60 examples/test_chunk_speed2 - 1073741824 $p 4194304 0 1 > gpurun_out/srv/ex_$p.log 2>&1 || exit 1
  PBS_SERVER_WGS=1 timeout -k 10 60 examples/test_chunk_speed2 - 1073741824 $p 4194304 0 1 > gpurun_out/srv/ex_${p}_w1.log 2>&1 || exit 1
done
