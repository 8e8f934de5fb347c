#!/bin/bash
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/gl8k
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gl8k/tests.log 2>&1
timeout -k 10 300 python3 bench.py --config c4 --alt-methods "" --walk-bytes 0 --api-bytes 0 > gpurun_out/gl8k/c4.json 2> gpurun_out/gl8k/c4.err
timeout -k 10 200 python3 bench.py --chunk 16384 --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --walk-bytes 0 > gpurun_out/gl8k/c16k.json 2> gpurun_out/gl8k/c16k.err
timeout -k 10 200 python3 bench.py --chunk 1024 --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --walk-bytes 0 > gpurun_out/gl8k/c1k.json 2> gpurun_out/gl8k/c1k.err
