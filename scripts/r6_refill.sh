#!/bin/bash
# k_encode's input refill with and without the compaction beside it:
# FETCH_SIZE per k_encode dispatch at AMBC_NSEG=4 (default) and 1 (no
# compaction concurrent with any encode), and kernel stats at NSEG=1
set -e
export TMPDIR=/tmp
O=gpurun_out/${EV_OUT:-r6refill}
mkdir -p $O
H="python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods= --walk-bytes 0 --ref-walk-bytes 0 --ref-full-walk-bytes 0 --no-verify --steps 2 --warmup 1"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch4 -o run -- $H > $O/fetch4.log 2>&1
AMBC_NSEG=1 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch1 -o run -- $H > $O/fetch1.log 2>&1
AMBC_NSEG=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats1 -o run -- $H > $O/stats1.log 2>&1
echo ok
