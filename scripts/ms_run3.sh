#!/bin/bash
# walk round: GPU walk tests, groups x walks x speculation sweep (second call timed),
# trace + kernel stats of the {1,2,3,4,5} walk
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "multisize or like_reference or host_scored" > gpurun_out/ms_tests.log 2>&1
rm -f gpurun_out/ms_sweep.log
for G in 1 2; do
  export AMBC_MS_GROUPS=$G
  echo "groups=$G" >> gpurun_out/ms_sweep.log
  CFGS="${CFGS:-2 512;3 512;2 1024 262144;3 1024 262144;2 2048 131072}" bash scripts/ms_sweep.sh
done
unset AMBC_MS_GROUPS
MS=1,2,3,4,5 TAG=ms5 bash scripts/ms_prof.sh
