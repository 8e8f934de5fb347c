#!/bin/bash
# per-segment statistics fused into k_compact (lib_fused = this tree) vs separate k_stats (lib_new8)
set -e
export TMPDIR=/tmp
O=gpurun_out/ssab2
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
for r in 1 2 3; do
  for L in new8 ss; do
    AMBC_LIB=ab/lib_$L.so timeout -k 10 200 python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --walk-bytes 0 --steps 10 --warmup 3 > $O/${L}_$r.json 2> $O/${L}_$r.err
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --walk-bytes 0 --no-verify --steps 3 --warmup 1 > $O/trace.log 2>&1
