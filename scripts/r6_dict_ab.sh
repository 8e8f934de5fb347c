#!/bin/bash
# same-box A/B of a k_dict variant (libambc_hip_exp.so, EXPFLAGS given at build)
# on the {1,2,3,4} leg (the reference's bytes), then the Dictionary GPU tests on it
set -e
O=gpurun_out/${EV_OUT:-r6dab2}
mkdir -p $O
B="python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --walk-bytes 0 --ref-walk-bytes 0 --ref-full-walk-bytes 0 --steps 3 --warmup 1 --alt-methods 1,2,3,4 --no-verify"
for r in 1 2; do
  timeout -k 10 300 $B > $O/base_$r.json 2> $O/base_$r.err
  AMBC_LIB=$PWD/adaptive-compression_amd/ambc/libambc_hip_exp.so timeout -k 10 300 $B > $O/exp_$r.json 2> $O/exp_$r.err
done
AMBC_LIB=$PWD/adaptive-compression_amd/ambc/libambc_hip_exp.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dict.py tests/test_gpu_dictany.py > $O/tests_exp.log 2>&1
echo ok
