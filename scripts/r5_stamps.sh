#!/bin/bash
# k_encode phase split (s_memtime stamps, diagnostic library), current code
set -e
export TMPDIR=/tmp
O=gpurun_out/r5st
mkdir -p $O
AMBC_STAMPS=1 AMBC_LIB=adaptive-compression_amd/ambc/libambc_hip_stamps.so timeout -k 10 200 \
    python3 scripts/kbench.py --msets "1,3,4,9" --inputs zero,random,ascii,mixed --reps 1 > $O/stamps.log 2>&1
echo stamps ok
