#!/bin/bash
# same-box A/B of a zlib-9 variant (libambc_hip_exp.so, EXPFLAGS given at build):
# {1,3,4,5z} leg and like_reference() walk, then the zlib-9 / walk GPU tests on it
set -e
O=gpurun_out/${EV_OUT:-r6z9ab}
mkdir -p $O
B="python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --walk-bytes 0 --ref-full-walk-bytes 0 --ref-walk-check-bytes 0 --steps 2 --warmup 1 --alt-methods 1,3,4,5z --no-verify"
for r in 1 2; do
  timeout -k 10 300 $B > $O/base_$r.json 2> $O/base_$r.err
  AMBC_LIB=$PWD/adaptive-compression_amd/ambc/libambc_hip_exp.so timeout -k 10 300 $B > $O/exp_$r.json 2> $O/exp_$r.err
done
AMBC_LIB=$PWD/adaptive-compression_amd/ambc/libambc_hip_exp.so timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_zlib9.py tests/test_gpu_walk.py tests/test_gpu_parity.py -k "zlib9 or z9 or like_reference or walk or deflate" > $O/tests_exp.log 2>&1
echo ok
