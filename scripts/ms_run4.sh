#!/bin/bash
# walk round: GPU walk tests, a sweep near the new defaults, {1,3,4,9} and {1,2,3,4,5} profiles
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_zlib9.py -m gpu -x -v --timeout 200 --timeout-method thread -k "multisize or like_reference or host_scored or gdeflate" > gpurun_out/ms_tests.log 2>&1
rm -f gpurun_out/ms_sweep.log
CFGS="3 1024 262144;4 1024 262144;3 2048 131072;4 2048 131072" bash scripts/ms_sweep.sh
echo "methods 1,2,3,4,5" >> gpurun_out/ms_sweep.log
MS=1,2,3,4,5 CFGS="2 1024 262144;3 1024 262144;2 512" bash scripts/ms_sweep.sh
bash scripts/ms_prof.sh
MS=1,2,3,4,5 TAG=ms5 bash scripts/ms_prof.sh
