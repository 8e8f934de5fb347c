#!/bin/bash
# same-box A/B: k_z9_parse<4096> with 8 (default) vs 10 waves per chunk
# (libambc_hip_exp.so built with EXPFLAGS=-DAMBC_Z9_NW4096=10), {1,3,4,5z}
set -e
O=gpurun_out/${EV_OUT:-r6z9nw}
mkdir -p $O
B="python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --walk-bytes 0 --ref-walk-bytes 0 --ref-full-walk-bytes 0 --steps 2 --warmup 1 --alt-methods 1,3,4,5z --no-verify"
for r in 1 2; do
  timeout -k 10 300 $B > $O/base_$r.json 2> $O/base_$r.err
  AMBC_LIB=$PWD/adaptive-compression_amd/ambc/libambc_hip_exp.so timeout -k 10 300 $B > $O/exp_$r.json 2> $O/exp_$r.err
done
AMBC_LIB=$PWD/adaptive-compression_amd/ambc/libambc_hip_exp.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_zlib9.py > $O/tests_exp.log 2>&1
echo ok
