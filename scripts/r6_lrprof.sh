#!/bin/bash
# kernel stats of the like_reference() walk leg alone (64 MiB)
set -e
export TMPDIR=/tmp
O=gpurun_out/${EV_OUT:-r6lr}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o run -- python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods= --walk-bytes 0 --ref-full-walk-bytes 0 --no-verify --steps 1 --warmup 0 --size 268435456 > $O/p.log 2>&1
echo ok
