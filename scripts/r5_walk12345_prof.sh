#!/bin/bash
# kernel split of the {1,2,3,4,5} multi-size walk on 256 MiB
set -e
export TMPDIR=/tmp
O=gpurun_out/r5wp
mkdir -p $O
MS_SETS="mixed:1,2,3,4,5" AMBC_TRACE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 scripts/multisize_bench.py 256 > $O/walk.log 2>&1
echo ok
