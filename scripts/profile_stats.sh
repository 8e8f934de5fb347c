#!/bin/bash
# rocprofv3 kernel stats of the headline bench (no alt leg) and of the DEFLATE
# method-set leg, each in its own run so every kernel's average is one workload.
set -e
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_head -o run -- \
    python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" > gpurun_out/prof_head.json 2> gpurun_out/prof_head.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_defl -o run -- \
    python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --methods 1,3,4,5 > gpurun_out/prof_defl.json 2> gpurun_out/prof_defl.err
