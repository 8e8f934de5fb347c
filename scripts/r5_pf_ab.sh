#!/bin/bash
# LZ4 A/B: pf1 = next-round prefetch (kept), new = pf1 + whole-chunk L2 touch;
# parity suite on the new library first (pf1 = prefetch of the round's bytes only)
set -e
export TMPDIR=/tmp
O=gpurun_out/r5pf3
mkdir -p $O
L=$PWD/adaptive-compression_amd/ambc
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
echo tests ok
for rep in 1 2; do
  for lib in pf1 new; do
    f=$L/libambc_hip.so; [ $lib = old ] && f=$L/libambc_hip_old.so; [ $lib = pf1 ] && f=$L/libambc_hip_pf1.so
    AMBC_LIB=$f timeout -k 10 200 python3 -u scripts/kbench.py --msets "1;9;1,3,4,9" --inputs zero,random,ascii,mixed --reps 5 > $O/kbench_${lib}_$rep.log 2>&1
    AMBC_LIB=$f timeout -k 10 300 python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --walk-bytes 0 --ref-walk-bytes 0 --ref-full-walk-bytes 0 --steps 10 --warmup 3 > $O/bench_${lib}_$rep.json 2> $O/bench_${lib}_$rep.err
  done
done
echo ab ok
C1="TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum"
K="python3 scripts/kbench.py --size 536870912 --reps 1 --inputs zero,random,ascii,mixed --msets 1;9;1,3,4,9"
timeout -s KILL 300 rocprofv3 --pmc $C1 --output-format csv -d $O/kb_req -o run -- $K > $O/kb_req.log 2>&1
echo pmc ok
