#!/bin/bash
# LZ4 probe A/B: pf1 = committed (round bytes a round ahead, formed at issue),
# pf2 = raw words carried to the next round, pipe = pf2 + the next round's
# candidates and their bytes (-DAMBC_LZ4_PIPE).  GPU suite on pf2 and pipe first.
set -e
export TMPDIR=/tmp
O=gpurun_out/r5pipe
mkdir -p $O
L=$PWD/adaptive-compression_amd/ambc
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_pf2.log 2>&1
echo tests pf2 ok
AMBC_LIB=$L/libambc_hip_exp.so timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_pipe.log 2>&1
echo tests pipe ok
for rep in 1 2; do
  for lib in pf1 pf2 pipe; do
    f=$L/libambc_hip.so; [ $lib = pf1 ] && f=$L/libambc_hip_pf1.so; [ $lib = pipe ] && f=$L/libambc_hip_exp.so
    AMBC_LIB=$f timeout -k 10 200 python3 -u scripts/kbench.py --msets "1;9;1,3,4,9" --inputs zero,random,ascii,mixed --reps 5 > $O/kbench_${lib}_$rep.log 2>&1
    AMBC_LIB=$f timeout -k 10 300 python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --walk-bytes 0 --ref-walk-bytes 0 --ref-full-walk-bytes 0 --steps 10 --warmup 3 > $O/bench_${lib}_$rep.json 2> $O/bench_${lib}_$rep.err
  done
done
echo ab ok
