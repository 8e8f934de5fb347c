#!/bin/bash
# the any-length plugin kernels' GPU tests
set -e
O=gpurun_out/${EV_OUT:-r6any}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_anylen.py tests/test_gpu_dictany.py > $O/tests.log 2>&1
echo ok
