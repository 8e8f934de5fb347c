#!/bin/bash
# k_encode {1,3,4,9} same-box A/B: the round's first library, this one, and this
# one without the Huffman emission code (diagnostic, -DAMBC_EXP_NO_HUFF_EMIT)
set -e
export TMPDIR=/tmp
O=gpurun_out/r5c
mkdir -p $O
L=$PWD/adaptive-compression_amd/ambc
for rep in 1 2 3; do
  for lib in old new noemit; do
    f=$L/libambc_hip.so; [ $lib = old ] && f=$L/libambc_hip_old.so; [ $lib = noemit ] && f=$L/libambc_hip_exp.so
    AMBC_LIB=$f timeout -k 10 200 python3 -u scripts/kbench.py --msets "1,3,4,9" --inputs ascii,mixed --reps 5 > $O/kbench_${lib}_$rep.log 2>&1
  done
done
