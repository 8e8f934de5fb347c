#!/bin/bash
set -e
O=gpurun_out/${EV_OUT:-r6plug}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_anylen.py tests/test_gpu_dictany.py tests/test_gpu_dict.py tests/test_gpu_huffdec.py > $O/tests.log 2>&1
timeout -k 10 500 python3 -u scripts/dictany_time.py > $O/plugins.jsonl 2> $O/plugins.err
echo ok
