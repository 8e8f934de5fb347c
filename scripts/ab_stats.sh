#!/bin/bash
# GPU check of the per-segment statistics, then a same-box bench A/B against the
# previous library (ab/lib_prev.so: statistics after the last compaction).
set -e
export TMPDIR=/tmp
O=gpurun_out/stats
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -k "pipelined or golden or bodies_match" -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --no-verify --steps 10 --warmup 2 > $O/new_$r.json 2>/dev/null
  AMBC_LIB=ab/lib_prev.so timeout -k 10 200 python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --no-verify --steps 10 --warmup 2 > $O/prev_$r.json 2>/dev/null
done
