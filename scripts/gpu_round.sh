#!/bin/bash
# One GPU-box pass: GPU tests, the default bench line, rocprofv3 kernel stats of the
# headline bench.  Each step under its own time limit, chained so a failure stops it.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1
timeout -k 10 400 python3 -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_head -o run -- \
    python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" > gpurun_out/prof_head.json 2> gpurun_out/prof_head.err
