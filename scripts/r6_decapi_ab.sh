#!/bin/bash
# same-box A/B of the decode host API: output prefault by MADV_POPULATE_WRITE
# (default library) vs a byte per page (libambc_hip_exp.so, -DAMBC_EXP_NOPOPULATE)
set -e
O=gpurun_out/${EV_OUT:-r6dab}
mkdir -p $O
B="python3 -u bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --walk-bytes 0 --ref-walk-bytes 0 --ref-full-walk-bytes 0 --steps 2 --warmup 1 --alt-methods 1,3,4;1,3,4,5"
for r in 1 2; do
  timeout -k 10 300 $B > $O/base_$r.json 2> $O/base_$r.err
  AMBC_LIB=$PWD/adaptive-compression_amd/ambc/libambc_hip_exp.so timeout -k 10 300 $B > $O/exp_$r.json 2> $O/exp_$r.err
done
echo ok
