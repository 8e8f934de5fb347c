#!/bin/bash
set -e
export TMPDIR=/tmp
bash scripts/ab_oldnew.sh
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "multisize or like_reference or host_scored or bodies_match or golden" > gpurun_out/oldnew/tests.log 2>&1
