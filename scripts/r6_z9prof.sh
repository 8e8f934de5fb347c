#!/bin/bash
set -e
export TMPDIR=/tmp
O=gpurun_out/${EV_OUT:-r6zp}
mkdir -p $O
B="python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --walk-bytes 0 --ref-walk-bytes 0 --ref-full-walk-bytes 0 --steps 1 --warmup 0 --no-verify"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- $B --alt-methods "1,3,4,5z" > $O/prof.log 2>&1
echo prof ok
