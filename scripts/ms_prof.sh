#!/bin/bash
# Multi-size walk profile: walk timing breakdown (AMBC_TRACE) and rocprofv3 kernel
# stats of one 256 MiB walk with the reference's eight candidates.
#   MS={1,3,4,9} (default) TAG=r3 scripts/ms_prof.sh
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-ms}
MS=${MS:-1,3,4,9}
cat > gpurun_out/ms_one.py <<EOF
import sys, time
sys.path[:0] = ['scripts', 'adaptive-compression_amd', '.']
import multisize_bench as m, ambc
data = m.mixed(256 << 20, 7)
comp = ambc.AdaptiveCompressor(methods=($MS))
comp.CHUNK_SIZE_CANDIDATES = list(comp.REFERENCE_CHUNK_SIZE_CANDIDATES)
comp._adaptive_compress(data[:1 << 20])
for _ in range(2):
    t = time.perf_counter(); b = comp._adaptive_compress(data); dt = time.perf_counter() - t
    print('walk', round(dt, 4), 's', round(len(data) / dt / 1e9, 3), 'GB/s', len(b), flush=True)
EOF
AMBC_TRACE=1 timeout -k 10 200 python3 gpurun_out/ms_one.py > gpurun_out/${TAG}_trace.log 2>&1
[ -n "$NOPROF" ] && exit 0
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- \
    python3 gpurun_out/ms_one.py > gpurun_out/${TAG}_prof.log 2>&1
