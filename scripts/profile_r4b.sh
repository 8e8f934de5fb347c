#!/bin/bash
# Round-4 headline-only kernel stats and FETCH / WRITE passes (no alternative
# method-set leg: its k_encode launches would mix into the headline kernel's numbers)
set -e
export TMPDIR=/tmp
O=gpurun_out/r4p
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_stats -o run -- \
    python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --walk-bytes 0 --ref-walk-bytes 0 --steps 5 --warmup 2 > $O/prof_stats.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- \
    python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --walk-bytes 0 --ref-walk-bytes 0 --no-verify --steps 2 --warmup 1 > $O/pmc_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- \
    python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --walk-bytes 0 --ref-walk-bytes 0 --no-verify --steps 2 --warmup 1 > $O/pmc_write.log 2>&1
