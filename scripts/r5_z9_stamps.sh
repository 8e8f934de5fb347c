#!/bin/bash
# zlib-9 parse phase split at 4 KiB (s_memtime stamps, diagnostic library) and
# rocprof kernel stats of the {1,3,4,5z} leg
set -e
export TMPDIR=/tmp
O=gpurun_out/r5z9st
mkdir -p $O
AMBC_STAMPS=1 AMBC_LIB=adaptive-compression_amd/ambc/libambc_hip_stamps.so Z9_CHUNKS=4096 timeout -k 10 200 \
    python3 scripts/z9_stamps_ms.py > $O/stamps.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "1,3,4,5z" --walk-bytes 0 --ref-walk-bytes 0 --ref-full-walk-bytes 0 --steps 2 --warmup 1 > $O/prof.log 2>&1
echo ok
