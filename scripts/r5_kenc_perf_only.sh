#!/bin/bash
# k_encode A/B without the suite (base = committed, new = under test)
set -e
export TMPDIR=/tmp
O=gpurun_out/${AB_OUT:-r5po}
mkdir -p $O
L=$PWD/adaptive-compression_amd/ambc
for rep in 1 2; do
  for lib in base new; do
    f=$L/libambc_hip.so; [ $lib = base ] && f=$L/libambc_hip_base.so
    AMBC_LIB=$f timeout -k 10 200 python3 -u scripts/kbench.py --msets "1;9;1,3,4,9" --inputs zero,random,ascii,mixed --reps 5 > $O/kbench_${lib}_$rep.log 2>&1
    AMBC_LIB=$f timeout -k 10 300 python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods= --walk-bytes 0 --ref-walk-bytes 0 --ref-full-walk-bytes 0 --steps 10 --warmup 3 > $O/bench_${lib}_$rep.json 2> $O/bench_${lib}_$rep.err
  done
done
echo ab ok
