#!/bin/bash
# Round-6 configuration sweep: C4 (chunk 8192), C3 (chunk 1024 / 16384), C5
# decode-only, and the any-window Dictionary plugin's throughput
set -e
export TMPDIR=/tmp
O=gpurun_out/r6cfg
mkdir -p $O
B="python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods= --walk-bytes 0 --ref-walk-bytes 0 --ref-full-walk-bytes 0 --steps 10 --warmup 3"
timeout -k 10 300 $B --config c4 > $O/c4.json 2> $O/c4.err
timeout -k 10 300 $B --chunk 1024 > $O/c3_1024.json 2> $O/c3_1024.err
timeout -k 10 300 $B --chunk 16384 > $O/c3_16384.json 2> $O/c3_16384.err
timeout -k 10 400 python3 -u scripts/c5_decode.py > $O/c5.json 2> $O/c5.err
timeout -k 10 300 python3 -u scripts/dictany_time.py > $O/dictany.jsonl 2> $O/dictany.err
echo cfg ok
