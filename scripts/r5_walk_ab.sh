#!/bin/bash
# The multi-size walk started as the input arrives: GPU tests of the walk, then
# the walk legs same-box with the walk after the whole upload
# (AMBC_MS_UPLOAD_FIRST, the round-4 behaviour) and without, twice each, AMBC_TRACE
set -e
export TMPDIR=/tmp
O=gpurun_out/r5d
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "multisize or like_reference or host_scored" --timeout 120 --timeout-method thread > $O/tests.log 2>&1
for rep in 1 2; do
  for v in first arrive; do
    if [ $v = first ]; then export AMBC_MS_UPLOAD_FIRST=1; else unset AMBC_MS_UPLOAD_FIRST; fi
    AMBC_TRACE=1 timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --no-verify --size 268435456 --alt-methods "" --ref-full-walk-bytes 0 --steps 1 --warmup 1 > $O/walk_${v}_$rep.json 2> $O/walk_${v}_$rep.err
  done
done
