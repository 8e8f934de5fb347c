#!/bin/bash
# decode host API across the bench's legs (fresh outputs in a long process)
set -e
O=gpurun_out/${EV_OUT:-r6da}
mkdir -p $O
timeout -k 10 600 python3 -u bench.py --no-cpu-baseline --api-bytes 0 --walk-bytes 0 --ref-walk-bytes 0 --ref-full-walk-bytes 0 --steps 3 --warmup 1 > $O/bench.json 2> $O/bench.err
echo ok
