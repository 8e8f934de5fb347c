#!/bin/bash
# Round 5: the Huffman emitter -- parity tests on the new library, then a
# same-box A/B of k_encode per input class with {1,3,4} (Huffman wins text) and
# the headline's {1,3,4,9}: the previous library (libambc_hip_old.so) against this one.
set -e
export TMPDIR=/tmp
O=gpurun_out/r5_huff
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
for lib in old new; do
  if [ $lib = old ]; then L=adaptive-compression_amd/ambc/libambc_hip_old.so; else L=adaptive-compression_amd/ambc/libambc_hip.so; fi
  AMBC_LIB=$PWD/$L timeout -k 10 200 python3 -u scripts/kbench.py --msets "1,3,4;1,3,4,9" --inputs zero,random,ascii,mixed --reps 3 > $O/kbench_$lib.log 2>&1
done
AMBC_LIB=$PWD/adaptive-compression_amd/ambc/libambc_hip_old.so timeout -k 10 200 python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "1,3,4" --walk-bytes 0 --ref-walk-bytes 0 --ref-full-walk-bytes 0 > $O/bench_old.json 2> $O/bench_old.err
timeout -k 10 200 python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "1,3,4" --walk-bytes 0 --ref-walk-bytes 0 --ref-full-walk-bytes 0 > $O/bench_new.json 2> $O/bench_new.err
timeout -k 10 300 python3 -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --walk-bytes 0 --ref-walk-bytes 0 --no-verify > $O/bench_fullwalk.json 2> $O/bench_fullwalk.err
AMBC_TRACE=1 timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --no-verify --size 268435456 --alt-methods "" --ref-full-walk-bytes 0 --steps 1 --warmup 1 > $O/walktrace.json 2> $O/walktrace.err
