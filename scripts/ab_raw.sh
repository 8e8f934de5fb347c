#!/bin/bash
# Same-box A/B of the raw-in-place compaction (default) against raw payloads
# copied through the slots (AMBC_RAW_VIA_SLOT=1), interleaved; then the PMC
# traffic passes of the headline bench (each counter its own run).
set -e
export TMPDIR=/tmp
O=gpurun_out/raw
mkdir -p $O
B="--no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods '' --no-verify --steps 10 --warmup 2"
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --no-verify --steps 10 --warmup 2 > $O/inplace_$r.json 2>/dev/null
  AMBC_RAW_VIA_SLOT=1 timeout -k 10 200 python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --no-verify --steps 10 --warmup 2 > $O/slot_$r.json 2>/dev/null
done
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --no-verify --steps 2 --warmup 1 > $O/fetch.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --no-verify --steps 2 --warmup 1 > $O/write.log 2>&1
