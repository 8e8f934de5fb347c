#!/bin/bash
# GPU-box profiling of the headline bench for profiles/ (run from the repo root):
#   bench line, rocprofv3 kernel stats, and two PMC passes (FETCH_SIZE / WRITE_SIZE
#   cannot share a pass on gfx950).  Every GPU step under its own time limit.
set -e
R=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_stats -o run -- \
    python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --steps 3 --warmup 1 > gpurun_out/prof_stats.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- \
    python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --no-verify --steps 2 --warmup 1 > gpurun_out/pmc_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- \
    python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --no-verify --steps 2 --warmup 1 > gpurun_out/pmc_write.log 2>&1
find gpurun_out/prof_stats gpurun_out/pmc_fetch gpurun_out/pmc_write -name "*.csv" | head -20
