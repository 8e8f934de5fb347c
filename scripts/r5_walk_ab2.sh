#!/bin/bash
# the walk's input upload: after it (first), staged pieces beside the walk
# (staged), registered pages by DMA beside the walk (registered); 3 rounds each
set -e
export TMPDIR=/tmp
O=gpurun_out/r5e
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "arrives or like_reference_reproduces" --timeout 120 --timeout-method thread > $O/tests.log 2>&1
for rep in 1 2 3; do
  for v in first registered; do
    AMBC_MS_UPLOAD=$v timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --no-verify --size 268435456 --alt-methods "" --ref-full-walk-bytes 0 --steps 1 --warmup 1 > $O/walk_${v}_$rep.json 2> $O/walk_${v}_$rep.err
  done
done
