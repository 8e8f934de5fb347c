#!/bin/bash
# multi-size walk round: GPU tests of the walk, the default-set profile, a
# walks x speculation sweep, and walk timings of the other method sets
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "multisize or like_reference" > gpurun_out/ms_tests.log 2>&1
bash scripts/ms_prof.sh
CFGS="${CFGS:-2 512;3 512;2 1024 262144;3 1024 262144;4 1024 262144;2 2048 131072;4 2048 131072}" bash scripts/ms_sweep.sh
for ms in "1,2,3,4,5" "1,2,3,4"; do
  MS_SETS="mixed:$ms" timeout -k 10 300 python3 scripts/multisize_bench.py 256 >> gpurun_out/ms_sets.log 2>&1
done
MS_MODE=reference MS_SETS="mixed:1,2,3,4,5" timeout -k 10 300 python3 scripts/multisize_bench.py 64 >> gpurun_out/ms_sets.log 2>&1
