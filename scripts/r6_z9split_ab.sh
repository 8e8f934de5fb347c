#!/bin/bash
# same-box A/B of the zlib-9 two-stream segments: AMBC_Z9_ONESTREAM=1 (base: parse,
# trees and emission of a segment on one stream) against the default (the trees and
# emission of segment i beside the parse of i + 1); then the GPU tests that cover it
set -e
O=gpurun_out/${EV_OUT:-r6z9split}
mkdir -p $O
B="python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --walk-bytes 0 --ref-full-walk-bytes 0 --ref-walk-check-bytes 0 --steps 2 --warmup 1 --alt-methods 1,3,4,5z --ref-walk-bytes 0"
for r in 1 2; do
  AMBC_Z9_ONESTREAM=1 timeout -k 10 300 $B > $O/base_$r.json 2> $O/base_$r.err
  timeout -k 10 300 $B > $O/exp_$r.json 2> $O/exp_$r.err
done
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_zlib9.py tests/test_gpu_parity.py tests/test_gpu_walk.py > $O/tests_exp.log 2>&1
echo ok
