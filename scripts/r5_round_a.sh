#!/bin/bash
# Round 5 pass A: the GPU suite on this library; same-box A/Bs of the Huffman
# emitter (libambc_hip_old.so: the round's first commit) and of the zlib-9 pair
# path (libambc_hip_exp.so: built with -DAMBC_Z9_PAIRS=0); the walk legs' host
# breakdown (AMBC_TRACE); the full-set reference walk.  Each step under its own limit.
set -e
export TMPDIR=/tmp
O=gpurun_out/r5a
mkdir -p $O
L=$PWD/adaptive-compression_amd/ambc
set +e
timeout -k 10 700 python3 -u -m pytest tests -m gpu -q --maxfail=10 --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?
set -e
echo "tests rc=$rc"
# (test failures: go on measuring; a fault, abort or time limit: stop here)
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for lib in old new; do
  f=$L/libambc_hip.so; [ $lib = old ] && f=$L/libambc_hip_old.so
  AMBC_LIB=$f timeout -k 10 200 python3 -u scripts/kbench.py --msets "1,3,4;1,3,4,9" --inputs zero,random,ascii,mixed --reps 3 > $O/kbench_huff_$lib.log 2>&1
done
for lib in nopairs pairs; do
  f=$L/libambc_hip.so; [ $lib = nopairs ] && f=$L/libambc_hip_exp.so
  AMBC_LIB=$f timeout -k 10 200 python3 -u scripts/kbench.py --msets "1,3,4,5" --flags 2 --inputs zero,random,ascii,mixed --reps 3 > $O/kbench_z9_$lib.log 2>&1
done
for lib in nopairs pairs; do
  f=$L/libambc_hip.so; [ $lib = nopairs ] && f=$L/libambc_hip_exp.so
  AMBC_LIB=$f timeout -k 10 200 python3 -u scripts/kbench.py --chunk 65536 --size 134217728 --msets "5" --flags 2 --inputs random,ascii,mixed --reps 2 > $O/kbench_z9big_$lib.log 2>&1
  AMBC_LIB=$f timeout -k 10 300 python3 -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --api-bytes 0 --no-e2e --no-verify --alt-methods "" --walk-bytes 0 --ref-full-walk-bytes 0 > $O/refwalk_$lib.json 2> $O/refwalk_$lib.err
done
for br in 128 256 512; do
  AMBC_MS_BREADTH=$br timeout -k 10 300 python3 -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --api-bytes 0 --no-e2e --no-verify --alt-methods "" --walk-bytes 0 --ref-full-walk-bytes 0 > $O/refwalk_br$br.json 2> $O/refwalk_br$br.err
done
timeout -k 10 400 python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "1,3,4;1,3,4,5z" --walk-bytes 0 --ref-full-walk-bytes 0 > $O/bench.json 2> $O/bench.err
AMBC_TRACE=1 timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --no-verify --size 268435456 --alt-methods "" --ref-full-walk-bytes 0 --steps 1 --warmup 1 > $O/walktrace.json 2> $O/walktrace.err
timeout -k 10 300 python3 -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --walk-bytes 0 --ref-walk-bytes 0 --no-verify > $O/fullwalk.json 2> $O/fullwalk.err
