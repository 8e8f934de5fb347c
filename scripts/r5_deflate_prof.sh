#!/bin/bash
# kernel split of the {1,3,4,5} (GPU DEFLATE) and {1,2,3,4} legs
set -e
export TMPDIR=/tmp
O=gpurun_out/r5dp
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p1345 -o run -- python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "1,3,4,5" --walk-bytes 0 --ref-walk-bytes 0 --ref-full-walk-bytes 0 --steps 2 --warmup 1 > $O/p1345.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p1234 -o run -- python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "1,2,3,4" --walk-bytes 0 --ref-walk-bytes 0 --ref-full-walk-bytes 0 --steps 2 --warmup 1 > $O/p1234.log 2>&1
echo ok
