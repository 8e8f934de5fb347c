#!/bin/bash
# GPU check of the tiled segment scan, then a same-box bench A/B against hipCUB's
# look-back scan (AMBC_SCAN_CUB=1), interleaved, and a kernel trace of each.
set -e
export TMPDIR=/tmp
O=gpurun_out/scan
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -k "pipelined or golden or bodies_match or large" -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --no-verify --steps 10 --warmup 2 > $O/tiled_$r.json 2>/dev/null
  AMBC_SCAN_CUB=1 timeout -k 10 200 python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --no-verify --steps 10 --warmup 2 > $O/cub_$r.json 2>/dev/null
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --no-verify --steps 5 --warmup 2 > $O/prof.json 2> $O/prof.err
