#!/bin/bash
# Direct emission with a waiting look-back (AMBC_DIRECT_EMIT=<polls>) vs the slot path
set -e
export TMPDIR=/tmp
O=gpurun_out/de2
mkdir -p $O
AMBC_DIRECT_EMIT=200 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "bodies_match or golden_files_bit_exact" > $O/tests.log 2>&1
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --walk-bytes 0 --steps 10 --warmup 3 > $O/off_$r.json 2> $O/off_$r.err
  for w in 20 200 2000; do
    AMBC_DIRECT_EMIT=$w AMBC_TRACE_DE=1 timeout -k 10 200 python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --walk-bytes 0 --steps 10 --warmup 3 > $O/w${w}_$r.json 2> $O/w${w}_$r.err
  done
done
