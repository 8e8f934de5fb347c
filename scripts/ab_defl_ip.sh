#!/bin/bash
# k_deflate reading 4-8 KiB chunks in place (default) vs staged in LDS (AMBC_DEFLATE_LDS=1)
set -e
export TMPDIR=/tmp
O=gpurun_out/deflip
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_zlib9.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
for r in 1 2; do
  for c in 4096 8192; do
    AMBC_DEFLATE_LDS=1 timeout -k 10 200 python3 bench.py --methods 1,3,4,5 --chunk $c --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --walk-bytes 0 --steps 6 --warmup 2 > $O/lds_${c}_$r.json 2> $O/lds_${c}_$r.err
    timeout -k 10 200 python3 bench.py --methods 1,3,4,5 --chunk $c --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --walk-bytes 0 --steps 6 --warmup 2 > $O/ip_${c}_$r.json 2> $O/ip_${c}_$r.err
  done
done
