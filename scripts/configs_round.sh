#!/bin/bash
# C2 (full bench line), C3 chunk sweep and C5 decode-only on one MI355X
# (--no-c2: skip the C2 line when bench.py has just produced it)
set -e
mkdir -p gpurun_out
if [ "$1" != "--no-c2" ]; then
  timeout -k 10 400 python3 -u bench.py > gpurun_out/c2.json 2> gpurun_out/c2.err
fi
for c in 1024 8192 16384; do
  timeout -k 10 300 python3 -u bench.py --chunk $c --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" \
      > gpurun_out/c3_$c.json 2> gpurun_out/c3_$c.err
done
timeout -k 10 400 python3 -u scripts/c5_decode.py > gpurun_out/c5.json 2> gpurun_out/c5.err
