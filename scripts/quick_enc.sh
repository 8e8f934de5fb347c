#!/bin/bash
# Quick GPU check of an encoder change: parity tests of the encoders, then the
# per-class k_encode timings (scripts/kbench.py) and one bench line.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_reference_suite.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/quick_tests.log 2>&1
timeout -k 10 120 python3 scripts/kbench.py --msets "1,3,4,9" --reps 5 > gpurun_out/quick_kbench.log 2>&1
timeout -k 10 300 python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" > gpurun_out/quick_bench.json 2> gpurun_out/quick_bench.err
