#!/bin/bash
# GPU zlib-9 id 5: parity tests, then per-kernel times (rocprofv3) of kbench
# with AMBC_FLAG_ZLIB9 on the four input classes.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_zlib9.py -x -q --timeout 240 --timeout-method thread > gpurun_out/z9_tests.log 2>&1
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/kp_z9 -o run -- \
  python3 scripts/kbench.py --flags 2 --inputs "${INPUTS:-zero,random,ascii,mixed}" --msets "${MS:-5;1,3,4,5}" --reps 3 > gpurun_out/kp_z9.log 2>&1
AMBC_STAMPS=1 AMBC_LIB=adaptive-compression_amd/ambc/libambc_hip_stamps.so timeout -k 10 120 python3 scripts/kbench.py --flags 2 --inputs "${INPUTS:-zero,random,ascii,mixed}" --msets 5 --reps 1 > gpurun_out/z9_stamps.log 2>&1
