#!/bin/bash
# kernel trace of one multi-size walk leg (WM: its methods) with the host
# breakdown (AMBC_TRACE), headline shrunk to 256 MiB, one step
set -e
export TMPDIR=/tmp
T=${TAG:-walk}
mkdir -p gpurun_out
AMBC_TRACE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof -o run -- \
    python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --no-verify --size 268435456 --alt-methods 1,3,4 \
    --ref-walk-bytes 0 --walk-methods ${WM:-1,2,3,4,5} --steps 1 --warmup 1 > gpurun_out/${T}_prof.json 2> gpurun_out/${T}_prof.err
