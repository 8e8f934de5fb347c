#!/bin/bash
# Non-temporal payload / compaction accesses (this library) against plain ones
# (libambc_hip_exp.so, -DAMBC_NT=0): the headline step same-box, interleaved, and
# FETCH_SIZE / WRITE_SIZE of the whole call (separate --pmc passes)
set -e
export TMPDIR=/tmp
O=gpurun_out/r5f
mkdir -p $O
L=$PWD/adaptive-compression_amd/ambc
B="--no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods '' --walk-bytes 0 --ref-walk-bytes 0 --ref-full-walk-bytes 0"
for rep in 1 2 3; do
  for v in nt plain; do
    f=$L/libambc_hip.so; [ $v = plain ] && f=$L/libambc_hip_exp.so
    AMBC_LIB=$f timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --walk-bytes 0 --ref-walk-bytes 0 --ref-full-walk-bytes 0 --no-verify --steps 10 --warmup 3 > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err
  done
done
for v in nt plain; do
  f=$L/libambc_hip.so; [ $v = plain ] && f=$L/libambc_hip_exp.so
  for c in FETCH_SIZE WRITE_SIZE; do
    AMBC_LIB=$f timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/pmc_${v}_$c -o run -- \
      python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --walk-bytes 0 --ref-walk-bytes 0 --ref-full-walk-bytes 0 --no-verify --steps 2 --warmup 1 > $O/pmc_${v}_$c.log 2>&1
  done
done
