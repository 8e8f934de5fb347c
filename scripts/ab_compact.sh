#!/bin/bash
# GPU check of the 16-byte k_compact, then a same-box bench A/B against
# ab/lib_prev_compact.so (dword k_compact), interleaved, and a kernel trace.
set -e
export TMPDIR=/tmp
O=gpurun_out/cmp
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_distributed.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --no-verify --steps 10 --warmup 2 > $O/new_$r.json 2>/dev/null
  AMBC_LIB=ab/lib_prev_compact.so timeout -k 10 200 python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --no-verify --steps 10 --warmup 2 > $O/prev_$r.json 2>/dev/null
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --no-verify --steps 5 --warmup 2 > $O/prof.json 2> $O/prof.err
