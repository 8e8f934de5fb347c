#!/bin/bash
# same-box A/B: the walk batches without per-batch copies / fills (default library,
# the working tree) vs with them (libambc_hip_exp.so, the previous commit): walk
# legs, like_reference(), {1,2,3,4}; then the whole GPU suite on the default library
set -e
O=gpurun_out/${EV_OUT:-r6wblit}
mkdir -p $O
B="python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --ref-full-walk-bytes 0 --steps 2 --warmup 1 --alt-methods 1,2,3,4 --no-verify"
for r in 1 2 3; do
  timeout -k 10 300 $B > $O/new_$r.json 2> $O/new_$r.err
  AMBC_LIB=$PWD/adaptive-compression_amd/ambc/libambc_hip_exp.so timeout -k 10 300 $B > $O/old_$r.json 2> $O/old_$r.err
done
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/tests_new.log 2>&1
echo ok
