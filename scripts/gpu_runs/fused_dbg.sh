#!/bin/bash
# which part breaks config 2: the entry table (PBS_FUSED_NOFAST=1 off) or four helpers + three scanners (PBS_FUSED_HELPERS=7)
mkdir -p gpurun_out/fd
K="config2-8GiB-random-4M and not multi and not fused-static"
for v in "PBS_FUSED_NOFAST=1" "PBS_FUSED_HELPERS=7" "PBS_FUSED_NOFAST=1 PBS_FUSED_HELPERS=7" "X=1"; do
  env $v timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "$K" > "gpurun_out/fd/$(echo $v | tr ' =' '__').log" 2>&1
  echo "$v rc=$?"
done
