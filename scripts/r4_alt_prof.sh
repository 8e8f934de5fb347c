#!/bin/bash
# round 4: kernel stats of the byte-pinned alt legs ({1,3,4,5z}, {1,2,3,4}) and the
# walk legs' host/device breakdown (AMBC_TRACE)
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r4}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_alt_prof -o run -- \
    python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --walk-bytes 0 --ref-walk-bytes 0 \
    --alt-methods "1,3,4,5z;1,2,3,4" --steps 2 --warmup 1 > gpurun_out/${T}_alt_prof.json 2> gpurun_out/${T}_alt_prof.err
AMBC_TRACE=1 timeout -k 10 300 python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" \
    --ref-walk-bytes 0 --steps 2 --warmup 1 > gpurun_out/${T}_walk_trace.json 2> gpurun_out/${T}_walk_trace.err
