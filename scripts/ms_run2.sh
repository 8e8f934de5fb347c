#!/bin/bash
# walk tests incl. host-scored ids 6/7, then the walk profile of the default set
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "multisize or like_reference or host_scored" > gpurun_out/ms_tests.log 2>&1
bash scripts/ms_prof.sh
