#!/bin/bash
# k_deflate A/B on the {1,3,4,5} leg and the {1,2,3,4,5} walk leg; GPU suite on new first
set -e
export TMPDIR=/tmp
O=gpurun_out/${AB_OUT:-r5dw}
mkdir -p $O
L=$PWD/adaptive-compression_amd/ambc
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_new.log 2>&1
echo tests new ok
for rep in 1 2; do
  for lib in base new; do
    f=$L/libambc_hip.so; [ $lib = base ] && f=$L/libambc_hip_base.so
    AMBC_LIB=$f timeout -k 10 400 python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "1,3,4,5" --ref-walk-bytes 0 --ref-full-walk-bytes 0 --steps 3 --warmup 1 > $O/bench_${lib}_$rep.json 2> $O/bench_${lib}_$rep.err
  done
done
echo ab ok
