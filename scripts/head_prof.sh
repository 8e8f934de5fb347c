#!/bin/bash
# rocprofv3 kernel trace + stats of the headline step alone (no walk legs)
set -e
export TMPDIR=/tmp
T=${TAG:-head}
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof -o run -- \
    python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --walk-bytes 0 --ref-walk-bytes 0 --alt-methods 1,3,4 \
    --steps 5 --warmup 2 > gpurun_out/${T}_prof.json 2> gpurun_out/${T}_prof.err
