#!/bin/bash
# Parity of the pass-A skip (chunks only LZ4 may take), then a same-box A/B against
# ab/lib_prev.so at chunk 16384 (C3), 8192 (C4's chunk: pass A without RLE's
# pair count and samples) and on the multi-size walk ({1,3,4,9}).
set -e
export TMPDIR=/tmp
O=gpurun_out/pa
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --chunk 16384 --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --no-verify --steps 6 --warmup 2 > $O/new16_$r.json 2>/dev/null
  AMBC_LIB=ab/lib_prev.so timeout -k 10 200 python3 bench.py --chunk 16384 --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --no-verify --steps 6 --warmup 2 > $O/prev16_$r.json 2>/dev/null
  timeout -k 10 200 python3 bench.py --chunk 8192 --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --no-verify --steps 6 --warmup 2 > $O/new8_$r.json 2>/dev/null
  AMBC_LIB=ab/lib_prev.so timeout -k 10 200 python3 bench.py --chunk 8192 --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --no-verify --steps 6 --warmup 2 > $O/prev8_$r.json 2>/dev/null
  MS_SETS="mixed:1,3,4,9" timeout -k 10 200 python3 scripts/multisize_bench.py 256 > $O/newms_$r.jsonl 2>/dev/null
  MS_SETS="mixed:1,3,4,9" AMBC_LIB=ab/lib_prev.so timeout -k 10 200 python3 scripts/multisize_bench.py 256 > $O/prevms_$r.jsonl 2>/dev/null
done
