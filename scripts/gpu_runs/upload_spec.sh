#!/bin/bash
# upload path: blobs encoded beside the copies (PBS_UPLOAD_SPEC=1, default) vs after the digests (0): tests, then the three bench stages each way
set -o pipefail
mkdir -p gpurun_out/up
NOEXTRA="--cpu-baseline 0 --cpu-config1 0 --host-inclusive-gib 0 --secondary-random 0"
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_digest.py -m gpu -k "upload or pipeline" > gpurun_out/up/tests.log 2>&1 || exit 1
for sp in 1 0; do
  PBS_UPLOAD_SPEC=$sp timeout -k 10 300 python bench.py --steps 2 --warmup 1 $NOEXTRA --upload-gib 64 > gpurun_out/up/vm_$sp.log 2>&1 || exit 1
  PBS_UPLOAD_SPEC=$sp timeout -k 10 300 python bench.py --steps 2 --warmup 1 $NOEXTRA --upload-gib 16 --upload-corpus text > gpurun_out/up/text_$sp.log 2>&1 || exit 1
done
PBS_UPLOAD_SPEC=1 timeout -k 10 300 python bench.py --steps 2 --warmup 1 $NOEXTRA --upload-gib 16 --upload-corpus pxar > gpurun_out/up/pxar_1.log 2>&1 || exit 1
