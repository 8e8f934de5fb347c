#!/bin/bash
# Round 6: the zlib-9 "cannot win" decision before the parse -- its tests and the
# {1,3,4,5z} bench leg, with a kernel trace of the leg
set -e
export TMPDIR=/tmp
O=gpurun_out/${EV_OUT:-r6z}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_zlib9.py -x -q --timeout 300 --timeout-method thread > $O/z9_tests.log 2>&1
echo z9 tests ok
B="python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --walk-bytes 0 --ref-full-walk-bytes 0 --steps 3 --warmup 1"
timeout -k 10 600 $B --alt-methods "1,3,4,5z" > $O/bench.json 2> $O/bench.err
echo bench ok
