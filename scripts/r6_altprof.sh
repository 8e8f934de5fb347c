#!/bin/bash
# kernel stats of the {1,2,3,4} (the reference's bytes) and {1,3,4,5} legs
set -e
export TMPDIR=/tmp
O=gpurun_out/${EV_OUT:-r6alt}
mkdir -p $O
for m in 1,2,3,4 1,3,4,5; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_${m//,/} -o run -- python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods= --walk-bytes 0 --ref-walk-bytes 0 --ref-full-walk-bytes 0 --no-verify --steps 3 --warmup 1 --methods $m > $O/p_${m//,/}.log 2>&1
done
echo ok
