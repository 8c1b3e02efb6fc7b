#!/bin/bash
# smoke -> gpu tests -> short bench; stops on any crash/timeout (exit codes other than
# 0 or 1 from pytest), never retries.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -m pytest tests -m gpu -x -q -k "not slow" > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --size-gib 8 --steps 5 --warmup 1 --cpu-baseline 0 --host-inclusive-gib 1 > gpurun_out/bench8.log 2>&1
rc=$?; echo "bench rc=$rc"; exit $rc
