#!/bin/bash
# the any-window Dictionary encoder's GPU tests (+ the batched Dictionary tests)
set -e
O=gpurun_out/${EV_OUT:-r6dany}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_dictany.py tests/test_gpu_dict.py > $O/tests.log 2>&1
echo ok
