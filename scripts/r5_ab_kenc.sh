#!/bin/bash
# k_encode same-box A/B: this library, the same with the Huffman tree not kept from
# the sizing merges (libambc_hip_exp.so, -DAMBC_HUFF_TREE_KEEP=0), and the round's
# first library (libambc_hip_old.so); interleaved, three times each; then the
# zlib-9 GPU tests and the headline bench line.
set -e
export TMPDIR=/tmp
O=gpurun_out/r5b
mkdir -p $O
L=$PWD/adaptive-compression_amd/ambc
for rep in 1 2 3; do
  for lib in old keep nokeep; do
    f=$L/libambc_hip.so; [ $lib = old ] && f=$L/libambc_hip_old.so; [ $lib = nokeep ] && f=$L/libambc_hip_exp.so
    AMBC_LIB=$f timeout -k 10 200 python3 -u scripts/kbench.py --msets "1,3,4;1,3,4,9" --inputs random,ascii,mixed --reps 3 > $O/kbench_${lib}_$rep.log 2>&1
  done
done
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_zlib9.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 400 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "1,3,4;1,3,4,5z" --walk-bytes 0 --ref-full-walk-bytes 0 > $O/bench.json 2> $O/bench.err
