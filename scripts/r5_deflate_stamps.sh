#!/bin/bash
# k_deflate phase split on the {1,3,4,5} workload (stamps library), per class
set -e
export TMPDIR=/tmp
O=gpurun_out/r5ds
mkdir -p $O
AMBC_STAMPS=1 AMBC_LIB=adaptive-compression_amd/ambc/libambc_hip_stamps.so timeout -k 10 200 \
    python3 scripts/kbench.py --msets "1,3,4,5" --inputs zero,random,ascii,mixed --reps 1 > $O/stamps.log 2>&1
echo ok
