#!/bin/bash
# Direct emission (AMBC_DIRECT_EMIT) vs the slot path: parity of the bodies, a
# same-box alternating bench A/B, and whole-call FETCH / WRITE traffic of both.
set -e
export TMPDIR=/tmp
O=gpurun_out/de
mkdir -p $O
AMBC_DIRECT_EMIT=1 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "bodies_match or golden_files_bit_exact or decisions_match" > $O/tests.log 2>&1
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --walk-bytes 0 --steps 10 --warmup 3 > $O/off_$r.json 2> $O/off_$r.err
  AMBC_DIRECT_EMIT=1 AMBC_TRACE_DE=1 timeout -k 10 200 python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --walk-bytes 0 --steps 10 --warmup 3 > $O/on_$r.json 2> $O/on_$r.err
done
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_off -o run -- python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --walk-bytes 0 --no-verify --steps 2 --warmup 1 > $O/fetch_off.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_off -o run -- python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --walk-bytes 0 --no-verify --steps 2 --warmup 1 > $O/write_off.log 2>&1
export AMBC_DIRECT_EMIT=1
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_on -o run -- python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --walk-bytes 0 --no-verify --steps 2 --warmup 1 > $O/fetch_on.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_on -o run -- python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --walk-bytes 0 --no-verify --steps 2 --warmup 1 > $O/write_on.log 2>&1
