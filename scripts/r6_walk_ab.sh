#!/bin/bash
# same-box A/B of a variant (libambc_hip_exp.so) on the multi-size walk legs
# ({1,3,4,9}, {1,2,3,4,5}) and the {1,2,3,4} leg, then the walk / Dictionary GPU tests on it
set -e
O=gpurun_out/${EV_OUT:-r6wab}
mkdir -p $O
B="python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --ref-walk-bytes 0 --ref-full-walk-bytes 0 --steps 2 --warmup 1 --alt-methods 1,2,3,4 --no-verify"
for r in 1 2 3; do
  timeout -k 10 300 $B > $O/base_$r.json 2> $O/base_$r.err
  AMBC_LIB=$PWD/adaptive-compression_amd/ambc/libambc_hip_exp.so timeout -k 10 300 $B > $O/exp_$r.json 2> $O/exp_$r.err
done
AMBC_LIB=$PWD/adaptive-compression_amd/ambc/libambc_hip_exp.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dict.py tests/test_gpu_walk.py > $O/tests_exp.log 2>&1
echo ok
