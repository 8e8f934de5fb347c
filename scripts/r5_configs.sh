#!/bin/bash
# Round-5 configuration sweep: C4 (chunk 8192), C3 (chunk 1024 / 16384), one line each
set -e
export TMPDIR=/tmp
O=gpurun_out/r5cfg
mkdir -p $O
B="python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods= --walk-bytes 0 --ref-walk-bytes 0 --ref-full-walk-bytes 0 --steps 10 --warmup 3"
timeout -k 10 300 $B --config c4 > $O/c4.json 2> $O/c4.err
timeout -k 10 300 $B --chunk 1024 > $O/c3_1024.json 2> $O/c3_1024.err
timeout -k 10 300 $B --chunk 16384 > $O/c3_16384.json 2> $O/c3_16384.err
echo cfg ok
