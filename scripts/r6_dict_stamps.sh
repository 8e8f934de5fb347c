#!/bin/bash
# k_dict phase split (s_memtime stamps, diagnostic library) and per-class times, {1,2,3,4}
set -e
export TMPDIR=/tmp
O=gpurun_out/${EV_OUT:-r6dst}
mkdir -p $O
AMBC_STAMPS=1 AMBC_LIB=adaptive-compression_amd/ambc/libambc_hip_stamps.so timeout -k 10 200 \
    python3 scripts/kbench.py --msets "1,2,3,4" --inputs ascii,mixed --reps 1 > $O/stamps.log 2>&1
timeout -k 10 200 python3 scripts/kbench.py --msets "1,3,4;1,2,3,4" --inputs zero,random,ascii,mixed --reps 3 > $O/kbench.log 2>&1
echo ok
