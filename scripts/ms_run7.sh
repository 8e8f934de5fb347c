#!/bin/bash
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/ms7
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "multisize or like_reference or host_scored" > gpurun_out/ms7/tests.log 2>&1
NOPROF=1 MS=1,3,4,9 TAG=ms7a bash scripts/ms_prof.sh
