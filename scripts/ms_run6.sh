#!/bin/bash
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/ms6
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "multisize or like_reference or host_scored" > gpurun_out/ms6/tests.log 2>&1
timeout -k 10 400 python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --steps 3 --warmup 1 > gpurun_out/ms6/bench.json 2> gpurun_out/ms6/bench.err
