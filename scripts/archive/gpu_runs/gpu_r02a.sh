#!/bin/bash
# Round 2, first GPU run: the GPU tests (new: reference digest vectors, periodic dense
# input, config 5 at full size), the default bench line (nproc CPU baseline, config 1 on
# the CPU), and the N=2 launcher refusing a 1-GPU box.  Each GPU step has its own limit.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp; O=gpurun_out/r02a; mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step pytest_gpu 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread || exit 1
step bench64 400 python bench.py || exit 1
python bench.py --gpus 2 --steps 1 > $O/bench_gpus2.log 2>&1; echo "gpus2 rc=$? (2 expected)"
echo done
