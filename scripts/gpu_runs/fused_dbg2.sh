#!/bin/bash
mkdir -p gpurun_out/fd
for v in "X=1" "PBS_FUSED=1" "PBS_DIRECT_OUT=0" "PBS_FUSED_HELPERS=7 PBS_FUSED_NOFAST=1"; do
  env $v timeout -k 10 120 python scripts/debug/fused_check.py 1 1 4194304 > "gpurun_out/fd/chk_$(echo $v | tr ' =' '__').log" 2>&1
  echo "$v rc=$? $(grep -h 'OK\|MISMATCH' gpurun_out/fd/chk_$(echo $v | tr ' =' '__').log | cut -c1-300)"
done
